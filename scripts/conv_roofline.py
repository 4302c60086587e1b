#!/usr/bin/env python
"""Per-kernel roofline of the ResNet-18 (bs512) 3x3 stride-1 convolutions.

For every (layer, pass) at the committed tuner pick it times, interleaved in one
process (cdna_hip_programming.md §5.4 rule 24):

* ``full``  -- the extension's kernel (what the training step runs);
* ``abl0``  -- the same kernel from the ablation library built with
  DMP_ABLATE=0 (must match ``full``: the library is a faithful copy);
* ``fill``  -- DMP_ABLATE=1: every global->LDS DMA of the kernel, no MFMA;
* ``mfma``  -- DMP_ABLATE=2: the MFMA work (and epilogue) on the first staged
  tile, no further DMA;
* ``noepi`` -- DMP_ABLATE=3: everything but the epilogue (halo fwd / dgrad);
* ``nolds`` -- DMP_ABLATE=4: the fragment reads of the MFMA loop removed
  (halo fwd / dgrad; the wgrad kernels are unchanged in 3 and 4);
* ``epirow`` -- not an ablation: the row-staged epilogue (DMP_HALO_EPI_LDS=1)
  on every halo forward too (the extension uses it for the data gradient);

and the fill ceiling of the chip (a DMA-only microkernel streaming 1-KiB
``buffer_load ... lds`` pieces per wave from an L2-resident and an HBM-sized
window).  Reported per kernel: achieved TF/s and share of the 2.5 PF dense
bf16 peak, bytes staged global->LDS (analytic, from the kernel's geometry),
achieved fill GB/s per CU and B/clk/CU at 2.4 GHz, and the fill / MFMA
ablation times as shares of the full kernel.

    python scripts/conv_roofline.py            (builds the ablation libraries if missing)
"""
import ctypes
import json
import math
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
CSRC = ROOT / "distributed_ml_pytorch_amd" / "csrc"
LIBDIR = ROOT / "distributed_ml_pytorch_amd" / "_ablate"
PEAK = 2.5e15
CLK = 2.4e9
CUS = 256

import torch  # noqa: E402

CL = torch.channels_last


def build_libs(force=False):
    LIBDIR.mkdir(exist_ok=True)
    srcs = [CSRC / "conv.hip", CSRC / "conv_wgrad.hip", CSRC / "ablate" / "ablate_entry.hip"]
    hdrs = list(CSRC.glob("*.h"))
    procs = []
    for n in (0, 1, 2, 3, 4, 5):
        out = LIBDIR / f"abl{n}.so"
        if not force and out.exists() and all(out.stat().st_mtime > s.stat().st_mtime
                                              for s in srcs + hdrs):
            continue
        # 5: not an ablation -- the candidate row-staged halo epilogue (DMP_HALO_EPI_LDS)
        flags = ["-DDMP_ABLATE=0", "-DDMP_HALO_EPI_LDS=1"] if n == 5 else [f"-DDMP_ABLATE={n}"]
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-std=c++17", "--offload-arch=gfx950",
               "-shared", *flags, "-I", str(CSRC), *map(str, srcs),
               "-Wl,--no-undefined", "-o", str(out)]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE))
    for p in procs:
        _, err = p.communicate()
        if p.returncode:
            raise RuntimeError(err.decode()[-3000:])


# ----------------------------------------------------------- staged-byte models
HALO = {0: (256, 64, 32, 4, 2, 2), 1: (128, 64, 32, 2, 2, 2), 2: (64, 64, 32, 2, 2, 2),
        3: (128, 64, 32, 4, 2, 2), 4: (256, 64, 32, 2, 2, 2), 5: (128, 64, 32, 2, 2, 1),
        6: (256, 64, 32, 4, 2, 1), 7: (64, 64, 32, 2, 2, 1), 8: (128, 64, 32, 4, 2, 1),
        9: (256, 64, 32, 4, 1, 1), 10: (256, 64, 32, 4, 1, 2), 11: (128, 64, 32, 2, 1, 1),
        12: (128, 128, 32, 2, 2, 1), 13: (256, 128, 32, 4, 2, 1), 14: (512, 64, 32, 8, 1, 1)}
HALOP = {115: (256, 2, 4), 116: (128, 3, 4), 117: (256, 2, 8)}
WH_NS = [2, 3, 4, 2, 3, 2, 2, 3]
WH_TR = [1, 1, 1, 3, 3, 1, 1, 1]
WH_PG = [1, 1, 1, 1, 1, 2, 1, 1]


def _tile_rows(bm, H, W):
    img = H * W
    if bm <= img:
        return bm // W, 1
    return H, bm // img


def bytes_halo(cfg, B, H, W, C, CO):
    """conv_halo_kernel: per block and chunk, the halo rows + 9 weight taps."""
    bm, bn, bk, wm, wn, ns = HALO[cfg - 100]
    th, tb = _tile_rows(bm, H, W)
    rpi = 64 // (bk // 8)
    a_ins = math.ceil(tb * (th + 2) * (W + 2) / rpi)
    stage = (a_ins * rpi * bk + 9 * bn * bk) * 2
    blocks = math.ceil(B * H * W / bm) * math.ceil(CO / bn)
    return blocks * (C // bk) * stage, blocks


def bytes_halop(cfg, B, H, W, C, CO):
    """conv_halo64p_kernel: resident weights once per block + every halo tile."""
    bm, ns, nw = HALOP[cfg]
    th, tb = _tile_rows(bm, H, W)
    ains = math.ceil(tb * (th + 2) * (W + 2) / 8)
    ntiles = math.ceil(B * H * W / bm)
    ny = CO // 64
    gx = min(math.ceil(CUS / ny), ntiles)
    return gx * ny * 9 * 64 * 64 * 2 + ntiles * ny * ains * 1024, gx * ny


def bytes_wgrad_halo(cfg, B, H, W, CI, CO):
    """conv_wgrad_halo_kernel: per (ci, co, tap-row) block and pixel tile, the dY
    tile + the shifted X rows."""
    if cfg >= 3000:
        cfg -= 2000
    idx = cfg - 1000
    var, rest = idx // 12, idx % 12
    bm = 224 if var >= 6 else 64 << (rest // 4)
    tr, pg = WH_TR[var], WH_PG[var]
    th, tb = _tile_rows(bm, H, W)
    thx = th + tr - 1
    xrows = tb * thx * (W + 2)
    xpw = math.ceil(math.ceil(xrows / 8) / (4 * pg))
    tile = bm * 64 * 2 + xpw * 4 * pg * 1024
    ntiles = math.ceil(B * H * W / bm)
    per = (CI // 64) * (CO // 64) * (3 // tr)
    return per * ntiles * tile, per


def staged_bytes(op, cfg, B, CI, H, W, CO):
    C_in, C_out = (CI, CO) if op == "fwd" else (CO, CI)
    if op == "wgrad":
        return bytes_wgrad_halo(cfg, B, H, W, CI, CO)
    if cfg in HALOP:
        return bytes_halop(cfg, B, H, W, C_in, C_out)
    if 100 <= cfg < 115:
        return bytes_halo(cfg, B, H, W, C_in, C_out)
    return None, None


# --------------------------------------------------------------------- timing
def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return 1e3 * a.elapsed_time(b) / iters        # us


def main():
    build_libs()
    from distributed_ml_pytorch_amd.ops._ext import native

    nat = native()
    libs = {n: ctypes.CDLL(str(LIBDIR / f"abl{n}.so")) for n in (0, 1, 2, 3, 4, 5)}
    for lib in libs.values():
        for fn in ("abl_conv_fwd", "abl_conv_dgrad", "abl_conv_wgrad", "abl_dma_ceiling"):
            getattr(lib, fn).restype = ctypes.c_int
        lib.abl_wgrad_slab_elems.restype = ctypes.c_longlong
    tune = json.load(open(ROOT / "tuning" / "mi355x_tune_cache.json"))
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = ctypes.c_void_p

    def ptr(t):
        return P(t.data_ptr())

    print("== fill ceiling (DMA-only microkernel, 1 block per CU)", flush=True)
    src = torch.empty(1 << 30, dtype=torch.uint8, device="cuda").random_(0, 255)
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    ceil = {}
    for window in (1 << 20, 1 << 30):
        for nw, inf in ((4, 8), (4, 16), (8, 8), (8, 16)):
            iters = 400
            us = timeit(lambda: libs[0].abl_dma_ceiling(ptr(src), ctypes.c_ulonglong(window), CUS,
                                                         nw, inf, iters, ptr(sink), stream), 5)
            byts = CUS * nw * inf * 1024 * iters
            gbs = byts / us / 1e3
            ceil[(window, nw, inf)] = gbs / CUS
            print(f"  window {window >> 20:5d} MiB  {nw} waves x {inf:2d} KiB in flight: "
                  f"{gbs / 1e3:6.2f} TB/s = {gbs / CUS:6.1f} GB/s/CU = "
                  f"{gbs * 1e9 / CUS / CLK:5.1f} B/clk/CU", flush=True)
    del src

    layers = [  # (name, B, CI, H, W, CO)
        ("s1 64ch 32x32", 512, 64, 32, 32, 64),
        ("s2 128ch 16x16", 512, 128, 16, 16, 128),
        ("s3 256ch 8x8", 512, 256, 8, 8, 256),
        ("s4 512ch 4x4", 512, 512, 4, 4, 512),
    ]
    print("\n== per kernel (us; interleaved rounds, median of 3)", flush=True)
    hdr = (f"{'layer':16s} {'pass':5s} {'cfg':>5s} {'full':>7s} {'abl0':>7s} {'fill':>7s} "
           f"{'mfma':>7s} {'noepi':>7s} {'nolds':>7s} {'epirow':>7s} {'TF/s':>6s} {'%peak':>5s} {'MB stg':>7s} {'GB/s/CU':>7s} "
           f"{'B/clk':>5s} {'fill%':>5s} {'mfma%':>5s}")
    print(hdr, flush=True)
    rows = []
    for name, B, CI, H, W, CO in layers:
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(B, CI, H, W, device="cuda", generator=g).to(torch.bfloat16).contiguous(
            memory_format=CL)
        w = (torch.randn(CO, CI, 3, 3, device="cuda", generator=g) * 0.05).to(
            torch.bfloat16).contiguous(memory_format=CL)
        wt = w.permute(1, 2, 3, 0).contiguous()
        dy = torch.randn(B, CO, H, W, device="cuda", generator=g).to(torch.bfloat16).contiguous(
            memory_format=CL)
        dw = torch.zeros(CO, CI, 3, 3, device="cuda").contiguous(memory_format=CL)
        part = torch.zeros(2 * 64 * max(CI, CO) + 4, device="cuda")
        y = torch.empty_like(dy)
        dx = torch.empty_like(x)
        flop = 2.0 * B * H * W * CO * CI * 9
        for op in ("fwd", "dgrad", "wgrad"):
            key = {"fwd": [op, B, CI, H, W, CO, 3, 3, 1, 1],
                   "dgrad": [op, B, CO, H, W, CI, H, W, 3, 3, 1, 1],
                   "wgrad": [op, B, CI, H, W, CO, CI, 3, 3, 1, 1]}[op]
            cfg = tune.get(json.dumps(key))
            if cfg is None:
                continue
            slab = None
            if op == "wgrad":
                se = libs[0].abl_wgrad_slab_elems(cfg, B, H, W, CI, CO, 3, 3, 1, 1)
                slab = torch.empty(max(int(se), 1), device="cuda")

            def full():
                if op == "fwd":
                    nat.conv_fwd(x, w, 1, 1, True, cfg)
                elif op == "dgrad":
                    nat.conv_dgrad(dy, w, H, W, 1, 1, cfg)
                else:
                    nat.conv_wgrad(dy, x, dw, 1, 1, cfg)

            def lib_fn(n):
                lib = libs[n]
                if op == "fwd":
                    return lambda: lib.abl_conv_fwd(ptr(x), ptr(w), ptr(y), ptr(part), B, H, W, CI,
                                                    H, W, CO, 3, 3, 1, 1, cfg, stream)
                if op == "dgrad":
                    return lambda: lib.abl_conv_dgrad(ptr(dy), ptr(wt), ptr(dx), B, H, W, CI, H,
                                                      W, CO, 3, 3, 1, 1, cfg, stream)
                return lambda: lib.abl_conv_wgrad(ptr(dy), ptr(x), ptr(dw), B, H, W, CI, H, W, CO,
                                                  3, 3, 1, 1, cfg,
                                                  ptr(slab) if slab is not None and slab.numel() > 1
                                                  else P(0), stream)

            arms = {"full": full, "abl0": lib_fn(0), "fill": lib_fn(1), "mfma": lib_fn(2),
                    "noepi": lib_fn(3), "nolds": lib_fn(4), "epirow": lib_fn(5)}
            ts = {k: [] for k in arms}
            for _ in range(3):
                for k, fn in arms.items():
                    ts[k].append(timeit(fn))
            med = {k: sorted(v)[1] for k, v in ts.items()}
            check = None
            if op in ("fwd", "dgrad"):
                # the candidate epilogue must reproduce the extension's output (and
                # the forward's BN partial sums)
                check = []
                for cand in (5,):
                    if op == "fwd":
                        ref, rpart, _ = nat.conv_fwd(x, w, 1, 1, True, cfg)
                        part.zero_()
                        lib_fn(cand)()
                        got = y
                        ps_ref = rpart[:2 * 64 * CO].view(2, 64, CO).sum(1)
                        ps_got = part[:2 * 64 * CO].view(2, 64, CO).sum(1)
                        pe = float((ps_ref - ps_got).abs().max() / ps_ref.abs().max())
                    else:
                        ref = nat.conv_dgrad(dy, w, H, W, 1, 1, cfg)
                        lib_fn(cand)()
                        got = dx
                        pe = 0.0
                    torch.cuda.synchronize()
                    check += [float((ref.float() - got.float()).norm() / ref.float().norm()), pe]
            byts, blocks = staged_bytes(op, cfg, B, CI, H, W, CO)
            tfs = flop / med["full"] / 1e6
            gbcu = (byts / med["full"] / 1e3 / CUS) if byts else float("nan")
            r = dict(layer=name, op=op, cfg=cfg, **{k: round(v, 2) for k, v in med.items()},
                     tflops=round(tfs, 1), pct_peak=round(100 * tfs * 1e12 / PEAK, 1),
                     staged_mb=round(byts / 1e6, 1) if byts else None, blocks=blocks,
                     gb_s_cu=round(gbcu, 1), b_clk_cu=round(gbcu * 1e9 / CLK, 1),
                     epirow_check=check,
                     fill_share=round(100 * med["fill"] / med["full"], 1),
                     mfma_share=round(100 * med["mfma"] / med["full"], 1))
            rows.append(r)
            print(f"{name:16s} {op:5s} {cfg:5d} {med['full']:7.1f} {med['abl0']:7.1f} "
                  f"{med['fill']:7.1f} {med['mfma']:7.1f} {med['noepi']:7.1f} {med['nolds']:7.1f} {med['epirow']:7.1f} {tfs:6.0f} {r['pct_peak']:5.1f} "
                  f"{r['staged_mb'] or 0:7.1f} {gbcu:7.1f} {r['b_clk_cu']:5.1f} "
                  f"{r['fill_share']:5.1f} {r['mfma_share']:5.1f}"
                  + (f"  err row {check[0]:.1e}/{check[1]:.1e}" if check else ""), flush=True)
    print("\nJSON " + json.dumps({"ceiling_gb_s_cu": {f"{k[0] >> 20}MiB_{k[1]}w_{k[2]}k": round(v, 1)
                                                      for k, v in ceil.items()},
                                  "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
