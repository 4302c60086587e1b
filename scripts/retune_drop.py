"""Drop tune-cache entries (JSON keys) that match every given substring, so the
next run re-tunes them against the current candidate lists.

    python scripts/retune_drop.py CACHE '3, 3, 1, 1]' '14, 14|7, 7'
('|' separates alternatives inside one pattern.)"""
import json
import sys


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    c = json.load(open(path))
    drop = [k for k in c if all(any(alt in k for alt in p.split("|")) for p in pats)]
    for k in drop:
        print("drop", k, c.pop(k))
    json.dump(c, open(path, "w"), indent=0, sort_keys=True)


if __name__ == "__main__":
    main()
