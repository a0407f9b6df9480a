"""Per-(kernel, grid) durations from a rocprofv3 kernel trace: the bench's dominant kernels run at several batch
sizes (act over B episodes, training launches over M, evaluation over 50), and the plain --stats average mixes
them.  usage: python3 tools/r04/kernel_by_grid.py <run_kernel_trace.csv> <out.csv> [kernel:workgroups]
With the optional marker only the launches that start before the marker's first launch count (e.g.
mpnn_forward_dense3_kernel:50, the first evaluation launch: the train bench's timed region and warmup, before its
untimed costs and learn_loop run concurrent evaluations)."""
import collections
import csv
import sys


def main(src, dst, marker=None):
    recs = []
    for r in csv.DictReader(open(src)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("eco::", "").strip()
        g = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        recs.append((n, g, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    stop = None
    if marker:
        mk, mg = marker.rsplit(":", 1)
        stop = min(t0 for n, g, t0, _ in recs if n == mk and g == int(mg))
    d = collections.defaultdict(list)
    for n, g, t0, t1 in recs:
        if stop is None or t0 < stop:
            d[(n, g)].append((t1 - t0) / 1e3)
    rows = sorted(d.items(), key=lambda kv: -sum(kv[1]))
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "workgroups", "calls", "avg_us", "min_us", "max_us", "total_ms"])
        for (n, g), v in rows:
            w.writerow([n, g, len(v), round(sum(v) / len(v), 2), round(min(v), 2), round(max(v), 2),
                        round(sum(v) / 1e3, 3)])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
