#!/usr/bin/env python
"""Same-process A/B of conv kernels between two source revisions.

``python scripts/conv_ab.py build <git-rev>`` (CPU): compiles conv.hip +
conv_wgrad.hip + csrc/ablate/ablate_entry.hip of the working tree and of
``<git-rev>`` into ``distributed_ml_pytorch_amd/_ablate/ab_{new,old}.so``
(ctypes entry points, never part of the extension).
``python scripts/conv_ab.py build-defines "-DX=0" "-DX=1"`` (CPU): both from the
working tree, old / new with the given compile-time flags.
``python scripts/conv_ab.py run [cfg ...]`` (GPU): times fwd / dgrad / wgrad of the
ResNet-18 bs512 3x3 layers with both libraries in interleaved rounds in ONE
process (median of CONV_AB_ROUNDS=9 rounds x 20 calls, alternating order) and checks that the two produce
bit-identical outputs (wgrad: equal to 1e-5, its split-K sums are fp32
atomics).  Default cfgs: the committed tuner picks per layer."""
import ctypes
import json
import os
import shutil
import statistics
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "distributed_ml_pytorch_amd" / "csrc"
LIBDIR = ROOT / "distributed_ml_pytorch_amd" / "_ablate"
SRCS = ["conv.hip", "conv_wgrad.hip"]
ROUNDS = int(os.environ.get("CONV_AB_ROUNDS", "9"))


def _compile(srcdir: Path, out: Path, defines=()):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-std=c++17", "--offload-arch=gfx950",
           "-shared", "-DDMP_ABLATE=0", *defines, "-I", str(srcdir),
           *[str(srcdir / s) for s in SRCS], str(srcdir / "ablate" / "ablate_entry.hip"),
           "-Wl,--no-undefined", "-o", str(out)]
    return subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)


def build(rev: str):
    LIBDIR.mkdir(exist_ok=True)
    tmp = Path(tempfile.mkdtemp(prefix="conv_ab_"))
    (tmp / "ablate").mkdir()
    for f in CSRC.glob("*.h"):
        rel = f"distributed_ml_pytorch_amd/csrc/{f.name}"
        txt = subprocess.run(["git", "show", f"{rev}:{rel}"], cwd=ROOT, capture_output=True)
        (tmp / f.name).write_bytes(txt.stdout if txt.returncode == 0 else f.read_bytes())
    for s in SRCS + ["ablate/ablate_entry.hip"]:
        rel = f"distributed_ml_pytorch_amd/csrc/{s}"
        txt = subprocess.run(["git", "show", f"{rev}:{rel}"], cwd=ROOT, capture_output=True,
                             check=True)
        (tmp / s).write_bytes(txt.stdout)
    procs = [_compile(CSRC, LIBDIR / "ab_new.so"), _compile(tmp, LIBDIR / "ab_old.so")]
    for p in procs:
        _, err = p.communicate()
        if p.returncode:
            raise SystemExit(err.decode()[-3000:])
    shutil.rmtree(tmp)
    print("built", LIBDIR / "ab_new.so", LIBDIR / "ab_old.so", f"(old = {rev})")


def build_defines(old_defs: str, new_defs: str):
    """Both libraries from the working tree, compiled with different -D flags."""
    LIBDIR.mkdir(exist_ok=True)
    procs = [_compile(CSRC, LIBDIR / "ab_new.so", new_defs.split()),
             _compile(CSRC, LIBDIR / "ab_old.so", old_defs.split())]
    for p in procs:
        _, err = p.communicate()
        if p.returncode:
            raise SystemExit(err.decode()[-3000:])
    print("built", f"old: {old_defs!r}", f"new: {new_defs!r}")


def stride2_wgrad(libs, tune, P, stream):
    """The stride-2 3x3 weight gradients (first conv of stages 2-4)."""
    import torch

    CL = torch.channels_last
    for name, B, CI, H, CO in [("s2 64->128 /2", 512, 64, 32, 128), ("s3 128->256 /2", 512, 128, 16, 256),
                               ("s4 256->512 /2", 512, 256, 8, 512)]:
        OH = H // 2
        key = json.dumps(["wgrad", B, CI, H, H, CO, CI, 3, 3, 2, 1])
        if key not in tune:
            continue
        cfg = tune[key]
        g = torch.Generator(device="cuda").manual_seed(1)
        x = torch.randn(B, CI, H, H, device="cuda", generator=g).to(torch.bfloat16).contiguous(
            memory_format=CL)
        dy = torch.randn(B, CO, OH, OH, device="cuda", generator=g).to(torch.bfloat16).contiguous(
            memory_format=CL)
        n = libs["new"].abl_wgrad_slab_elems(cfg, B, H, H, CI, CO, 3, 3, 2, 1)
        slab = torch.empty(max(n, 1), device="cuda")
        outs = {k: torch.zeros(CO, CI, 3, 3, device="cuda").contiguous(memory_format=CL)
                for k in libs}

        def call(k):
            outs[k].zero_()
            return libs[k].abl_conv_wgrad(P(dy.data_ptr()), P(x.data_ptr()), P(outs[k].data_ptr()),
                                          B, H, H, CI, OH, OH, CO, 3, 3, 2, 1, cfg,
                                          P(slab.data_ptr() if n > 0 else 0), stream)
        for k in libs:
            assert call(k) == 0, (k, cfg)
        torch.cuda.synchronize()
        d = float((outs["old"] - outs["new"]).norm() / outs["old"].norm())
        times = {k: [] for k in libs}
        for rnd in range(ROUNDS):
            for k in (("old", "new") if rnd % 2 == 0 else ("new", "old")):
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(20):
                    call(k)
                b.record()
                b.synchronize()
                times[k].append(a.elapsed_time(b) / 20 * 1e3)
        to, tn = statistics.median(times["old"]), statistics.median(times["new"])
        print(f"{name:16s} {'wgrad':5s} {cfg:5d} {to:8.1f} {tn:8.1f} {100 * (tn / to - 1):+6.1f}%  "
              f"{'yes' if d < 1e-5 else 'NO':>7s}   min {min(times['old']):6.1f} "
              f"{min(times['new']):6.1f}", flush=True)


def run(cfgs_arg):
    sys.path.insert(0, str(ROOT))
    import torch

    libs = {k: ctypes.CDLL(str(LIBDIR / f"ab_{k}.so")) for k in ("old", "new")}
    for lib in libs.values():
        lib.abl_conv_fwd.restype = ctypes.c_int
        lib.abl_conv_dgrad.restype = ctypes.c_int
        lib.abl_conv_wgrad.restype = ctypes.c_int
        lib.abl_wgrad_slab_elems.restype = ctypes.c_longlong
    tune = json.load(open(ROOT / "tuning" / "mi355x_tune_cache.json"))
    P = ctypes.c_void_p
    stream = P(torch.cuda.current_stream().cuda_stream)
    CL = torch.channels_last
    layers = [("s1 64ch 32x32", 512, 64, 32, 32, 64), ("s2 128ch 16x16", 512, 128, 16, 16, 128),
              ("s3 256ch 8x8", 512, 256, 8, 8, 256), ("s4 512ch 4x4", 512, 512, 4, 4, 512)]
    print(f"{'layer':16s} {'pass':5s} {'cfg':>5s} {'old us':>8s} {'new us':>8s} {'delta':>7s}  bitwise"
          f"   (median of {ROUNDS} rounds x 20 calls; min)")
    stride2_wgrad(libs, tune, P, stream)
    for name, B, CI, H, W, CO in layers:
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(B, CI, H, W, device="cuda", generator=g).to(torch.bfloat16).contiguous(
            memory_format=CL)
        w = (0.05 * torch.randn(CO, CI, 3, 3, device="cuda", generator=g)).to(
            torch.bfloat16).contiguous(memory_format=CL)
        wt = w.permute(1, 2, 3, 0).contiguous()      # [CI][R][S][CO]
        dy = torch.randn(B, CO, H, W, device="cuda", generator=g).to(torch.bfloat16).contiguous(
            memory_format=CL)
        part = torch.zeros(2 * 64 * CO + 4, device="cuda")
        for op in ("fwd", "dgrad", "wgrad"):
            key = json.dumps([op, B, CI, H, W, CO, 3, 3, 1, 1]) if op == "fwd" else \
                json.dumps([op, B, CO, H, W, CI, H, W, 3, 3, 1, 1]) if op == "dgrad" else \
                json.dumps([op, B, CI, H, W, CO, CI, 3, 3, 1, 1])
            cfgs = [int(c) for c in cfgs_arg] or ([tune[key]] if key in tune else [])
            for cfg in cfgs:
                outs, times = {}, {k: [] for k in libs}
                slab = None
                for k, lib in libs.items():
                    if op == "wgrad":
                        outs[k] = torch.zeros(CO, CI, 3, 3, device="cuda").contiguous(
                            memory_format=CL)
                        n = lib.abl_wgrad_slab_elems(cfg, B, H, W, CI, CO, 3, 3, 1, 1)
                        if n > 0 and (slab is None or slab.numel() < n):
                            slab = torch.empty(n, device="cuda")
                        continue
                    out = torch.empty(B, CO if op == "fwd" else CI, H, W, device="cuda",
                                      dtype=torch.bfloat16).contiguous(memory_format=CL)
                    outs[k] = out

                def call(k):
                    if op == "wgrad":
                        outs[k].zero_()
                        return libs[k].abl_conv_wgrad(P(dy.data_ptr()), P(x.data_ptr()),
                                                      P(outs[k].data_ptr()), B, H, W, CI, H, W,
                                                      CO, 3, 3, 1, 1, cfg,
                                                      P(slab.data_ptr() if slab is not None
                                                        else 0), stream)
                    if op == "fwd":
                        part.zero_()
                        return libs[k].abl_conv_fwd(P(x.data_ptr()), P(w.data_ptr()),
                                                    P(outs[k].data_ptr()), P(part.data_ptr()), B,
                                                    H, W, CI, H, W, CO, 3, 3, 1, 1, cfg, stream)
                    return libs[k].abl_conv_dgrad(P(dy.data_ptr()), P(wt.data_ptr()),
                                                  P(outs[k].data_ptr()), B, H, W, CI, H, W, CO, 3,
                                                  3, 1, 1, cfg, stream)
                for k in libs:
                    assert call(k) == 0, (k, op, cfg)
                torch.cuda.synchronize()
                if op == "wgrad":   # fp32 atomics: equal up to summation order
                    d = (outs["old"] - outs["new"]).norm() / outs["old"].norm()
                    same = bool(d < 1e-5)
                else:
                    same = torch.equal(outs["old"], outs["new"])
                for rnd in range(ROUNDS):   # alternate which library goes first
                    for k in (("old", "new") if rnd % 2 == 0 else ("new", "old")):
                        a = torch.cuda.Event(enable_timing=True)
                        b = torch.cuda.Event(enable_timing=True)
                        a.record()
                        for _ in range(20):
                            call(k)
                        b.record()
                        b.synchronize()
                        times[k].append(a.elapsed_time(b) / 20 * 1e3)
                to, tn = statistics.median(times["old"]), statistics.median(times["new"])
                mo, mn = min(times["old"]), min(times["new"])
                print(f"{name:16s} {op:5s} {cfg:5d} {to:8.1f} {tn:8.1f} {100 * (tn / to - 1):+6.1f}%  "
                      f"{'yes' if same else 'NO':>7s}   min {mo:6.1f} {mn:6.1f} "
                      f"{100 * (mn / mo - 1):+5.1f}%", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "build":
        build(sys.argv[2])
    elif len(sys.argv) > 3 and sys.argv[1] == "build-defines":
        build_defines(sys.argv[2], sys.argv[3])
    elif len(sys.argv) > 1 and sys.argv[1] == "run":
        run(sys.argv[2:])
    else:
        raise SystemExit(__doc__)
