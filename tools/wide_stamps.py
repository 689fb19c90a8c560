"""Where the wide kernel's K loop spends its cycles (WQ4_WIDE_STAMP build):
per Large-V3 encoder shape at M = ROWS, the s_memtime cycles of waves 0 and
4 of every workgroup in the vmcnt waits, the barriers, the LDS-DMA issue and
the compute, as fractions of the loop, plus the loop's cycles per half step.

    WQ4_LIB_DIR=whisper-burn_amd/diag/stampw python tools/wide_stamps.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "whisper-burn_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))

import oracle  # noqa: E402
import wq4  # noqa: E402

M = int(os.environ.get("ROWS", "48000"))
SHAPES = [(3840, 1280), (1280, 1280), (5120, 1280), (1280, 5120)]


def main():
    L = wq4.lib()
    vp = ctypes.c_void_p
    st = vp(torch.cuda.current_stream().cuda_stream)
    L.wq4_debug_set_enc_kernel(5)
    rng = np.random.default_rng(0)
    for n, k in SHAPES:
        q = oracle.quantize_convert_np((rng.standard_normal(n * k) * 0.05).astype(np.float32))
        t = wq4.Q4Tensor.from_q4_bytes(q, [n, k], decode_step=False)
        x = torch.randn(M, k, device="cuda")
        at = torch.empty(L.wq4_atiled_bytes(M, k, 0), dtype=torch.uint8, device="cuda")
        wq4.check(L.wq4_tile_activations(vp(x.data_ptr()), M, k, k, 0, vp(at.data_ptr()), at.numel(), st))
        y = torch.empty(M, n, device="cuda")
        ms = []
        for _ in range(4):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            wq4.check(L.wq4_gemm_tiled(t.handle, None, vp(at.data_ptr()), None, vp(y.data_ptr()), None, M, 0, 0, 1, st))
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        mg, ng = (-(-M // 32) + 7) // 8, (n // 32 + 7) // 8
        wgs = min(mg * ng, 4096)
        buf = (ctypes.c_ulonglong * (wgs * 20))()
        got = L.wq4_diag_wide_stamps(buf, wgs)
        raw = np.frombuffer(buf, dtype=np.uint64).reshape(wgs, 2, 10)[:got]
        a = raw.astype(np.float64)
        tot = a[:, :, 4]
        halves = 2 * ((k // 32 + 1) // 2)
        for w, name in ((0, "wave 0"), (1, "wave 4")):
            fr = a[:, w, :4].sum(0) / tot[:, w].sum()
            print(f"N={n:5d} K={k:5d} {name}: vmcnt {fr[0]:.3f} barrier {fr[1]:.3f} issue {fr[2]:.3f} "
                  f"compute {fr[3]:.3f}; {np.median(tot[:, w]) / halves:7.0f} cycles per half step "
                  f"(compute {np.median(a[:, w, 3]) / halves:6.0f}); clock {np.median(tot[:, w] / a[:, w, 5]) * 0.1:.2f} GHz",
                  flush=True)
        # the whole launch against the K loops: rounds of one workgroup per CU
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        rounds = -(-mg * ng // cus)
        loop_us = np.median(a[:, 0, 5]) * 0.01
        kern_us = ms[-1] * 1e3
        print(f"N={n:5d} K={k:5d} launch {kern_us:7.1f} us = {rounds} rounds x {kern_us / rounds:5.1f} us; "
              f"K loop {loop_us:5.1f} us per workgroup (median), {kern_us / rounds - loop_us:5.1f} us per round outside it; "
              f"{2 * M * n * k / (kern_us * 1e-6) / 1e12:6.1f} TF/s", flush=True)
        # workgroup lifetimes (wave 0, absolute 100 MHz ticks): entry -> K loop
        # start -> K loop end -> epilogue stores complete; the CUs' occupancy
        ent = raw[:, 0, 6].astype(np.int64)
        end = raw[:, 0, 7].astype(np.int64)
        lp = a[:, 0, 5]
        life = (end - ent) * 0.01
        span = (end.max() - ent.min()) * 0.01
        if got == mg * ng:
            print(f"N={n:5d} K={k:5d} workgroup life {np.median(life):6.1f} us median = K loop {np.median(lp) * 0.01:6.1f}"
                  f" + the rest {np.median(life - lp * 0.01):5.1f} (prologue to loop + epilogue); "
                  f"CU occupancy {life.sum() / (cus * span):.3f} over the {span:.0f}-us span", flush=True)
            lend = raw[:, 0, 8].astype(np.int64)
            iss = raw[:, 0, 9].astype(np.int64)
            st0 = lend - (a[:, 0, 5]).astype(np.int64)
            print(f"N={n:5d} K={k:5d}   entry -> loop {np.median(st0 - ent) * 0.01:5.1f} us, loop end -> epilogue issued "
                  f"{np.median(iss - lend) * 0.01:5.1f} us, -> stores complete {np.median(end - iss) * 0.01:5.1f} us", flush=True)


if __name__ == "__main__":
    main()
