"""Achievable bf16 MFMA rate and sustained shader clock on this box (MI355X_MICROARCH.md
"DVFS give-back" items 1, 6, 7).  Diagnostics for bench.py's roofline (`peak_achievable`) and tools/clock_probe.py;
no training path imports this module.

`mfma_peak()` runs `scd_calib_mfma_peak` (16 independent v_mfma_f32_16x16x32_bf16 chains per wave on random bf16
operands held in registers, a different operand pair per instruction) back to back for `warm_s` seconds, so the chip
settles at the clock it holds under sustained MFMA load, then times `reps` launches with HIP events and reads the
in-kernel clock of the last one: Δs_memtime / Δs_memrealtime x 100 MHz per wave (median over waves).
"""
import statistics
import time

import torch

from . import lib as L
from . import ops

MFMA_FLOP = 2 * 16 * 16 * 32          # one v_mfma_f32_16x16x32_bf16


def cus():
    return torch.cuda.get_device_properties(0).multi_processor_count


def stamp_clock(stamps, n):
    """median shader clock (GHz) and median loop cycles over the first n records of a [n][4] int64 stamp buffer"""
    s = stamps[:n].cpu().tolist()
    ghz, cyc = [], []
    for t0, t1, r0, r1 in s:
        if r1 > r0 and t1 > t0:
            ghz.append((t1 - t0) / (r1 - r0) * 0.1)
            cyc.append(t1 - t0)
    if not ghz:
        return None, None
    return statistics.median(ghz), statistics.median(cyc)


def mfma_peak(waves_per_simd=2, warm_s=2.5, reps=10, target_ms=4.0, zeros=False):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(11)
    n = 256 * 8 * 64 * 8
    src = torch.zeros(n, device=dev, dtype=torch.bfloat16) if zeros else \
        (torch.rand(n, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    grid = cus() * waves_per_simd
    out = torch.empty(grid * 256, device=dev, dtype=torch.float32)
    stamps = torch.zeros(grid * 4 * 4, device=dev, dtype=torch.int64)

    def launch(iters, st=None):
        L.call("scd_calib_mfma_peak", ops.ptr(src), grid, iters, ops.ptr(out), ops.ptr(st) if st is not None else None,
               ops.stream())

    # size one launch to ~target_ms at ~2 GHz: 16 MFMAs x 16 cycles per iteration and wave, k waves per SIMD
    iters = max(64, int(target_ms * 1e-3 * 2.0e9 / (256 * waves_per_simd)))
    launch(iters)
    torch.cuda.synchronize()
    t_end = time.time() + warm_s
    while time.time() < t_end:
        for _ in range(8):
            launch(iters)
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps - 1):
        launch(iters)
    launch(iters, stamps)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    flop = grid * 4 * iters * 16 * MFMA_FLOP
    ghz, cyc = stamp_clock(stamps.view(-1, 4), grid * 4)
    return {"waves_per_simd": waves_per_simd, "operands": "zeros" if zeros else "random", "grid": grid,
            "iters": iters, "ms_per_launch": round(ms, 4), "tflops": round(flop / ms / 1e9, 1),
            "clock_ghz": round(ghz, 3) if ghz else None,
            "cycles_per_mfma_per_wave": round(cyc / (iters * 16), 2) if cyc else None,
            "tflops_at_2.4ghz": round(cus() * 4 * 1024 * 2.4e9 / 1e12, 1)}
