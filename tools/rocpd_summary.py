"""Summarise a rocprofv3 kernel-trace database (rocpd SQLite) without the rocpd tools.

    python tools/rocpd_summary.py gpurun_out/prof/run_results.db [--steps]

Prints per-kernel calls / avg / min / max / total (us) like `--stats`, and with --steps the
per-position timeline of one decode step of the last replay: kernel, grid, duration and the gap
to the previous kernel's end (what a persistent design would remove)."""
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sys.argv[1]
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, grid_x, workgroup_x, lds_size, vgpr_count, sgpr_count "
                     "from kernels order by start").fetchall()
    agg = defaultdict(list)
    for r in rows:
        agg[r[0]].append((r[2] - r[1]) / 1e3)
    print(f"{'kernel':70s} {'calls':>7s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s} {'total_ms':>9s}")
    for name, d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{name[:70]:70s} {len(d):7d} {sum(d) / len(d):9.3f} {min(d):9.3f} {max(d):9.3f} {sum(d) / 1e3:9.3f}")
    if "--steps" in sys.argv:
        # last step: from the last step_begin to the end
        idx = [i for i, r in enumerate(rows) if "step_begin" in r[0]]
        if len(idx) >= 2:
            a, b = idx[-2], idx[-1]
            print(f"\none step ({b - a} kernels), wall {(rows[b][1] - rows[a][1]) / 1e3:.1f} us")
            busy = 0.0
            gaps = 0.0
            for i in range(a, b):
                r = rows[i]
                gap = (r[1] - rows[i - 1][2]) / 1e3
                dur = (r[2] - r[1]) / 1e3
                busy += dur
                gaps += gap if i > a else 0.0
                if i - a < 12 or i >= b - 3:
                    print(f"  {r[0][:60]:60s} grid {r[3] // max(r[4], 1):5d}x{r[4]:4d} lds {r[5]:6d} "
                          f"vgpr {r[6]:3d} dur {dur:8.2f} gap {gap:6.2f}")
            print(f"  busy {busy:.1f} us, gaps {gaps:.1f} us")


if __name__ == "__main__":
    main()
