#!/usr/bin/env python3
"""K1a phase timeline from an NK_ABL_STAMPS build (tools/ab_build.sh abl_stamps
-DNK_ABL_STAMPS): runs config 2's step a few hundred times, then reads the last
launch's per-workgroup stamps (s_memtime at the phase barriers, s_memrealtime at
start/end, HW_ID/XCC_ID) and prints mean phase durations and residency.

    NK_AB_LIB=tools/bin/ab/abl_stamps/libneurokmer.so python tools/k1a_stamps.py
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from neurokmer_amd import SpikingKmerCounter, _lib, synth  # noqa: E402

PHASES = ["stage", "phase1 (window+hash+rank)", "scan+reserve", "sort", "write"]


def main():
    bases, offs = synth.make_records(115_000_000, 7, seed=synth.SEED, repeats_per_mb=64,
                                     motif_len=200)
    d_b = torch.from_numpy(bases).cuda()
    d_o = torch.from_numpy(offs.view(np.int64)).cuda()
    c = SpikingKmerCounter(31, 1.0, 0.95, 2, 1.0, 2_000_000, True)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    for _ in range(400):
        c.reset(s.cuda_stream, blocking=False)
        c.process_parallel_device(d_b.data_ptr(), d_o.data_ptr(), 7, bases.size, s.cuda_stream)
    torch.cuda.synchronize()
    L = _lib.load()
    n_tiles = (bases.size + 8191) // 8192
    L.nk_diag_stamps.argtypes = [C.c_void_p, C.c_size_t]
    buf = (C.c_ulonglong * (n_tiles * 16))()
    assert L.nk_diag_stamps(buf, n_tiles * 16) == 0
    st = np.frombuffer(buf, np.uint64).reshape(n_tiles, 16).astype(np.int64)
    hw = st[:, 1]
    d = np.diff(st[:, [8, 2, 3, 4, 5, 6]], axis=1)  # s_memtime deltas (shader clocks)
    real0, real1 = st[:, 0], st[:, 7]
    life_ns = (real1 - real0) * 10.0  # s_memrealtime: 100 MHz
    span_ns = (real1.max() - real0.min()) * 10.0
    out = {"tiles": int(n_tiles), "kernel_span_us": span_ns / 1e3,
           "wg_life_us_mean": float(life_ns.mean() / 1e3),
           "wg_life_us_p50": float(np.median(life_ns) / 1e3)}
    # phase durations in shader clocks (stage = start..2 is not stamped by
    # s_memtime at 0: use realtime start for the stage length instead)
    clk = {}
    for i, name in enumerate(PHASES):
        clk[name] = float(np.mean(d[:, i]))
        clk[name + " p90"] = float(np.percentile(d[:, i], 90))
    out["phase_clk_mean"] = clk
    # average residency: sum of lifetimes / span / CUs
    cu_key = (hw >> 32) * 4096 + (hw & 0xFFF)  # xcc, (se, sh, cu bits) of HW_ID
    n_cu = len(np.unique(cu_key))
    out["cus_seen"] = int(n_cu)
    out["mean_wg_resident_per_cu"] = float(life_ns.sum() / span_ns / max(n_cu, 1))
    # stage duration from realtime start to stamp 2 is not comparable (different
    # clocks); report the fraction of a WG's life spent in each phase via memtime
    # total = stamp6 - stamp2 plus the stage estimate life - (that)/clk
    tot = (st[:, 6] - st[:, 8]).astype(np.float64)
    out["sclk_ghz_est"] = float(np.median(tot / np.maximum(life_ns, 1)))
    out["wg_clk_mean"] = float(tot.mean())
    # concurrency over time: WGs alive per CU at 100 sample instants
    t = np.linspace(real0.min(), real1.max(), 100)
    alive = [(np.sum((real0 <= x) & (real1 > x))) / max(n_cu, 1) for x in t]
    out["alive_per_cu_timeline"] = [round(float(a), 2) for a in alive]
    out["note"] = "phase clocks are s_memtime deltas between the phase barriers (thread 0)"
    print(json.dumps(out, indent=1))
    c.close()


if __name__ == "__main__":
    main()
