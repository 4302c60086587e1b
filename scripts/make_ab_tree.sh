#!/bin/bash
# Build a second, self-contained copy of the framework at git revision REV into DIR
# (bench.py + package + tuning + its own in-tree extension), for whole-bench A/Bs of two
# revisions on one GPU box:  python DIR/bench.py ...  vs  python bench.py ...
#   bash scripts/make_ab_tree.sh HEAD~1 ab/old      (CPU; list DIR in nothing: it must travel)
set -e
REV=${1:?rev}; DIR=${2:?dir}
cd "$(dirname "$0")/.."
rm -rf "$DIR" && mkdir -p "$DIR"
git archive "$REV" bench.py distributed_ml_pytorch_amd tuning | tar -x -C "$DIR"
(cd "$DIR" && python -m distributed_ml_pytorch_amd._build > /dev/null)
ls -la "$DIR"/distributed_ml_pytorch_amd/_native*.so
