"""Per-(kernel, grid) durations from a rocprofv3 kernel trace: the bench's dominant kernels run at several batch
sizes (act over B episodes, training launches over M, evaluation over 50), and the plain --stats average mixes
them.  usage: python3 tools/r04/kernel_by_grid.py <run_kernel_trace.csv> <out.csv>"""
import collections
import csv
import sys


def main(src, dst):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(src)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("eco::", "").strip()
        g = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        d[(n, g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = sorted(d.items(), key=lambda kv: -sum(kv[1]))
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "workgroups", "calls", "avg_us", "min_us", "max_us", "total_ms"])
        for (n, g), v in rows:
            w.writerow([n, g, len(v), round(sum(v) / len(v), 2), round(min(v), 2), round(max(v), 2),
                        round(sum(v) / 1e3, 3)])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
