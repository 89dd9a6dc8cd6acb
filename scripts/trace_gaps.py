#!/usr/bin/env python
"""Kernel timeline of a rocprofv3 --kernel-trace database (rocpd SQLite): over the
last `--window` ms of dispatches, GPU busy fraction (union of kernel intervals),
the idle gaps between dependent kernels, and time per kernel class.
    trace_gaps.py <trace_results.db> [--window 100]
"""
import argparse
import re
import sqlite3
from collections import defaultdict

CLASSES = [("gemm256s_kernel", "gemm"), ("attention", "attention"), ("ln_stats", "ln_stats"),
           ("layernorm", "layernorm"), ("splitk", "cls_splitk"), ("q0", "attention_q0"),
           ("im2col", "im2col"), ("gemm", "gemm_other"), ("head", "head"), ("topk", "head")]


def kclass(name):
    for key, cls in CLASSES:
        if key in name:
            return cls
    return re.sub(r"\W.*", "", name)[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--window", type=float, default=100.0, help="ms at the end of the trace")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    q = ("select d.start, d.end, s.kernel_name from rocpd_kernel_dispatch d join "
         "rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start")
    ev = [(s, e, n) for s, e, n in c.execute(q)]
    t_end = max(e for _, e, _ in ev)
    t0 = t_end - a.window * 1e6
    ev = [x for x in ev if x[0] >= t0]
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e, _ in ev:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    wall = cur_e - ev[0][0]
    per = defaultdict(lambda: [0, 0.0])
    for s, e, n in ev:
        k = kclass(n)
        per[k][0] += 1
        per[k][1] += (e - s) / 1e6
    gaps.sort()
    print(f"window {wall / 1e6:.2f} ms, {len(ev)} dispatches, busy {busy / wall:.3f}, "
          f"idle {(wall - busy) / 1e6:.3f} ms in {len(gaps)} gaps "
          f"(median {gaps[len(gaps) // 2] / 1e3 if gaps else 0:.2f} us, "
          f"p90 {gaps[int(len(gaps) * 0.9)] / 1e3 if gaps else 0:.2f} us)")
    for k, (n, ms) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"  {k:14s} {n:6d} launches {ms:9.3f} ms  {ms / n * 1e3:8.2f} us avg")


if __name__ == "__main__":
    main()
