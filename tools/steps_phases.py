"""Per-phase timeline of the schedule form (k_bo_steps / k_lo_steps) at
config 2 from its device stamps (s_memrealtime, 100 MHz = 10 ns ticks):
median / p90 over the units of each phase's duration, the spread of unit
start times, and the kernel span.  python tools/steps_phases.py [bo|lo]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import tenstorrentallreduce_amd as t  # noqa: E402


def main():
    variant = t.LO if (len(sys.argv) > 1 and sys.argv[1] == "lo") else t.BO
    if len(sys.argv) > 2:   # key=value tune settings (A/B)
        for kv in sys.argv[2:]:
            k, v = kv.split("=")
            t.tune(k, int(v))
    side, total, n = 8, 64, 327680
    stride = t.preferred_rank_stride(n)
    buf = (torch.rand((total, stride), device="cuda:0") * 100).to(torch.bfloat16).view(torch.int16)
    plan = t.Plan(t.SWING, variant, side, n, total, t.EXEC_STEPS)
    st = torch.zeros(plan.stamp_words, dtype=torch.int64, device="cuda:0")
    for _ in range(20):
        plan.execute(buf.data_ptr(), stride, None, None, stamps_ptr=st.data_ptr())
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    plan.execute(buf.data_ptr(), stride, None, None, stamps_ptr=st.data_ptr())
    e1.record()
    torch.cuda.synchronize()
    S = 6
    per = 2 * S + 1 if variant == t.BO else S + 1
    u = st.cpu().numpy().view(np.uint64).reshape(-1, per).astype(np.int64)
    t0 = u[:, 0].min()
    d = np.diff(u, axis=1) * 10   # ns
    out = {"variant": "bo" if variant == t.BO else "lo", "tune": sys.argv[2:], "units": int(u.shape[0]),
           "kernel_us_events": round(e0.elapsed_time(e1) * 1e3, 2),
           "span_us_stamps": round((u[:, -1].max() - t0) / 100, 2),
           "unit_start_us": {"p50": round(float(np.median(u[:, 0] - t0)) / 100, 2),
                             "max": round(float((u[:, 0] - t0).max()) / 100, 2),
                             "late_over_3us": int(((u[:, 0] - t0) > 300).sum())},
           "unit_total_us_p50": round(float(np.median(u[:, -1] - u[:, 0])) / 100, 2),
           "phase_us_p50": [round(float(np.median(d[:, q])) / 1000, 3) for q in range(d.shape[1])],
           "phase_us_p90": [round(float(np.percentile(d[:, q], 90)) / 1000, 3) for q in range(d.shape[1])]}
    # k_steps_reg: unit u's stamps are those of wave 0 of workgroup u % grid, strip u // grid
    # of that wave (a persistent grid of `grid` workgroups): split by strip index
    grid = int(os.environ.get("STEPS_GRID", "0"))
    if grid:
        for j in range(int(np.ceil(u.shape[0] / grid))):
            sel = u[j * grid:(j + 1) * grid]
            dd = np.diff(sel, axis=1) * 10
            out[f"strip{j}"] = {"units": int(sel.shape[0]),
                                "start_us_p50_max": [round(float(np.median(sel[:, 0] - t0)) / 100, 2),
                                                     round(float((sel[:, 0] - t0).max()) / 100, 2)],
                                "end_us_p50_max": [round(float(np.median(sel[:, -1] - t0)) / 100, 2),
                                                   round(float((sel[:, -1] - t0).max()) / 100, 2)],
                                "step0_us_p50": round(float(np.median(dd[:, 0])) / 1000, 3),
                                "chain_us_p50": round(float(np.median(dd[:, 1:-1 if variant == t.BO else None].sum(axis=1))) / 1000, 3),
                                "stores_us_p50": round(float(np.median(dd[:, -1])) / 1000, 3) if variant == t.BO else None}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
