"""Per-queue busy fraction of a concurrent run (rocprofv3 --kernel-trace CSV): over the window from the first
k_load_values of the timed steps to the last kernel end, the union of each hardware queue's kernel intervals, the
time no queue runs anything, and which kernels occupy each queue. Shows which stream idles in a pipelined step.

python tools/queue_busy.py run_kernel_trace.csv [first_call [n_calls]]
   first_call: index of the first k_load_values of the window (skip the warm-up calls); n_calls: calls in the window
   (default: to the end), e.g. bench.py --steps 3 --warmup 1 with 4 calls per step: 4 12"""
import csv
import sys
from collections import defaultdict


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main(path, skip=2, ncalls=0):
    def bare(name):  # no return type, namespaces or arguments: k_emit_ect<0, 16>
        return name.split("(")[0].replace("void ", "").split("::")[-1]
    rows = sorted(((bare(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"])
                   for r in csv.DictReader(open(path))), key=lambda r: r[1])
    loads = [r[1] for r in rows if r[0].startswith("k_load_values")]
    if len(loads) <= skip:
        skip = 0
    t0 = loads[skip]
    t_end = loads[skip + ncalls] if ncalls and skip + ncalls < len(loads) else None
    win = [r for r in rows if r[1] >= t0 and r[0].startswith("k_") and (t_end is None or r[1] < t_end)]
    t1 = max(r[2] for r in win)  # the last kernel of the window (not the next call's start: host gaps)
    span = t1 - t0
    byq, byk = defaultdict(list), defaultdict(lambda: defaultdict(float))
    for name, s, e, q in win:
        byq[q].append((s, e))
        byk[q][name.split("<")[0]] += e - s
    print("window %.2f ms from call %d, %s calls (%d kernels)" % (span / 1e6, skip, ncalls or "all", len(win)))
    print("any queue busy: %.1f %%" % (100.0 * union([(s, e) for _, s, e, _ in win]) / span))
    for q in sorted(byq, key=lambda q: int(q) if q.isdigit() else 0):
        b = union(byq[q])
        top = sorted(byk[q].items(), key=lambda kv: -kv[1])[:4]
        print("queue %-3s busy %5.1f %%  %s" % (q, 100.0 * b / span,
                                               ", ".join("%s %.1f ms" % (k, v / 1e6) for k, v in top)))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2, int(sys.argv[3]) if len(sys.argv) > 3 else 0)
