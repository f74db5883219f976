"""Per-kernel launch counts and mean / median durations from rocprofv3 sqlite outputs (the
`--kernel-trace` default format on this image), one column per run directory; with --by-grid
the kernels are also split by grid size (e.g. the GEMM stages of one step)."""
import glob
import sqlite3
import statistics
import sys


def stats(d, by_grid):
    db = glob.glob(f"{d}/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    rows = c.execute("select name, grid_x, grid_y, end - start from kernels").fetchall()
    out = {}
    for name, gx, gy, dur in rows:
        key = (name[:70] + (f" [{gx}x{gy}]" if by_grid else ""))
        out.setdefault(key, []).append(dur / 1000.0)
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    by_grid = "--by-grid" in sys.argv
    runs = [stats(d, by_grid) for d in args]
    keys = sorted(set().union(*runs), key=lambda k: -sum(runs[0].get(k, [0])))
    for k in keys:
        cols = []
        for r in runs:
            v = r.get(k)
            cols.append(f"{len(v):6d} {statistics.mean(v):8.2f} {statistics.median(v):8.2f}" if v else " " * 24)
        print(" | ".join(cols), "|", k)


if __name__ == "__main__":
    main()
