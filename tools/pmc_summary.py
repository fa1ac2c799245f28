"""Per-kernel PMC summary (last dispatch of each kernel) from rocprofv3 counter_collection CSVs.

usage: pmc_summary.py DIR_PREFIX   (reads DIR_PREFIX_sq, _rd, _wr)
       pmc_summary.py DIR_PREFIX --json BATCH OUT.json [WORKLOAD [LAYOUT_KEY]]   (bench.py's config.workload and
       config.layout_key: "O0", or the --sym argument of a mapped line)
FETCH_SIZE is doubled (gfx950 reports half the bytes of wide streaming reads; MI355X_MICROARCH.md
HBM section); FETCH_SIZE / WRITE_SIZE are in KB."""
import csv
import os
import sys
from collections import defaultdict


def load(path):
    per = defaultdict(dict)  # (kernel, dispatch) -> counters
    dur = {}
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pzk::", "")
        key = (k, int(r["Dispatch_Id"]))
        per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    agg = defaultdict(lambda: defaultdict(float))
    n = defaultdict(int)
    for (k, d), c in per.items():
        n[k] += 1
        for name, v in c.items():
            agg[k][name] += v
        agg[k]["ms"] += dur[(k, d)]
    return {k: {name: v / n[k] for name, v in c.items()} for k, c in agg.items()}


def main(prefix):
    sq = load(prefix + "_sq/run_counter_collection.csv")
    rd = load(prefix + "_rd/run_counter_collection.csv") if os.path.exists(prefix + "_rd") else {}
    wr = load(prefix + "_wr/run_counter_collection.csv") if os.path.exists(prefix + "_wr") else {}
    print(f"{'kernel':26s} {'ms':>7s} {'waves':>9s} {'valu/wave':>9s} {'salu/w':>7s} {'vmwr/w':>7s} "
          f"{'lds/w':>6s} {'rd GB':>7s} {'wr GB':>7s} {'rd+wr GB/s':>10s}")
    for k in sorted(sq, key=lambda k: -sq[k]["ms"]):
        c = sq[k]
        w = max(c.get("SQ_WAVES", 1), 1)
        rgb = 2 * rd.get(k, {}).get("FETCH_SIZE", 0) * 1024 / 1e9
        wgb = wr.get(k, {}).get("WRITE_SIZE", 0) * 1024 / 1e9
        ms = wr.get(k, {}).get("ms", c["ms"])
        print(f"{k:26s} {c['ms']:7.3f} {w:9.0f} {c.get('SQ_INSTS_VALU', 0) / w:9.0f} {c.get('SQ_INSTS_SALU', 0) / w:7.0f} "
              f"{c.get('SQ_INSTS_VMEM_WR', 0) / w:7.1f} {c.get('SQ_INSTS_LDS', 0) / w:6.0f} {rgb:7.2f} {wgb:7.2f} "
              f"{(rgb + wgb) / ms if ms else 0:10.1f}")


def traffic_json(prefix, batch, out_path, workload=None, layout_key="O0"):
    """Per-kernel HBM traffic per witness (FETCH_SIZE x 2 + WRITE_SIZE, bytes) for bench.py's
    roofline.traffic; batch = witnesses per launch of the profiled run."""
    import json
    def bare(r):  # bare kernel name: no return type, template arguments or namespaces (pzk::ec_c1::k_...)
        return r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]

    def sums(path):
        tot, calls = defaultdict(lambda: defaultdict(float)), defaultdict(int)
        for r in csv.DictReader(open(path)):
            k = bare(r)
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[(k, r["Dispatch_Id"])] = 1
        return tot

    def durations(path):  # kernel -> summed dispatch duration (ms); the counter passes serialise dispatches
        dur = {}
        for r in csv.DictReader(open(path)):
            dur[(bare(r), r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        out = defaultdict(float)
        for (k, _), v in dur.items():
            out[k] += v
        return out
    rd = sums(prefix + "_rd/run_counter_collection.csv")
    wr = sums(prefix + "_wr/run_counter_collection.csv")
    # every batch launches k_load_values exactly once
    n_batches = len({r["Dispatch_Id"] for r in csv.DictReader(open(prefix + "_wr/run_counter_collection.csv"))
                     if "k_load_values" in r["Kernel_Name"]})
    # the instruction-mix pass (SQ_INSTS_VALU: wave-level VALU instructions) for the VALU roofline
    sq_path = prefix + "_sq/run_counter_collection.csv"
    sq, n_sq = {}, 0
    if os.path.exists(sq_path):
        sq = sums(sq_path)
        n_sq = len({r["Dispatch_Id"] for r in csv.DictReader(open(sq_path)) if "k_load_values" in r["Kernel_Name"]})
    ms = durations(prefix + "_wr/run_counter_collection.csv")
    res = {}
    valu_total = 0.0
    for k in sorted(set(rd) | set(wr) | set(sq)):
        if not k.startswith("k_"):
            continue
        f = 2 * rd.get(k, {}).get("FETCH_SIZE", 0) * 1024 / n_batches
        w = wr.get(k, {}).get("WRITE_SIZE", 0) * 1024 / n_batches
        res[k] = {"fetch_bytes_per_witness": round(f / batch), "write_bytes_per_witness": round(w / batch),
                  "traffic_bytes_per_witness": round((f + w) / batch),
                  "standalone_ms_per_batch": round(ms.get(k, 0.0) / n_batches, 4)}
        if n_sq:
            v = sq.get(k, {}).get("SQ_INSTS_VALU", 0) / n_sq / batch
            res[k]["valu_insts_per_witness"] = round(v, 1)
            valu_total += v
    out = {"source": prefix, "batch": batch, "workload": workload, "layout_key": layout_key, "kernels": res}
    if n_sq:
        out["valu_insts_per_witness"] = round(valu_total, 1)
    json.dump(out, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    if len(sys.argv) > 3 and sys.argv[2] == "--json":
        traffic_json(sys.argv[1], int(sys.argv[3]), sys.argv[4], sys.argv[5] if len(sys.argv) > 5 else None,
                     sys.argv[6] if len(sys.argv) > 6 else "O0")
    else:
        main(sys.argv[1])
