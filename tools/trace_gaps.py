"""Kernel timeline of the last timed step from a rocprofv3 --kernel-trace CSV:
per-kernel start offset, duration and the idle gap before it.

    python tools/trace_gaps.py gpurun_out/trace/.../run_kernel_trace.csv [--steps 3]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 3
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    rows.sort()
    # the bench's steps start with k_part_hist; take the last one
    starts = [i for i, r in enumerate(rows) if "k_part_hist" in r[2]]
    # a whole step from one k_part_hist to the next (the host's work between steps included), else
    # the last step to the end of the trace
    seg = rows[starts[-2]:starts[-1] + 1] if len(starts) >= 2 else rows[starts[-1]:]
    t0 = seg[0][0]
    prev_end = t0
    busy = gap = 0
    for s, e, name in seg:
        g = max(0, s - prev_end)
        busy += e - s
        gap += g
        print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {g / 1e3:7.1f}  {name[:70]}")
        prev_end = max(prev_end, e)
    print(f"step span {(prev_end - t0) / 1e3:.1f} us, kernels {busy / 1e3:.1f} us, gaps {gap / 1e3:.1f} us")


if __name__ == "__main__":
    main()
