"""VALU issue cycles per witness from one rocprofv3 counter pass (tools/gpu/gpu_pmc_valu.sh).

SQ_INSTS_VALU counts wave-level VALU instructions; SQ_ACTIVE_INST_VALU the quad-cycles waves spend executing them
(the counter behind rocprof's VALUBusy = SQ_ACTIVE_INST_VALU / CU_NUM / GRBM_GUI_ACTIVE). Their ratio is the mean
cycles a VALU instruction holds its SIMD: 64-bit integer multiply-adds and DPP moves are not single-issue, so
instruction counts alone understate how much of the chip's VALU a kernel takes.

usage: pmc_valu.py RUN_COUNTER_COLLECTION.csv BATCH [WITNESSES_PER_S [OUT.json]]
  BATCH: witnesses per launch of the profiled run; WITNESSES_PER_S (optional): a line's measured rate, for the
  job's VALU cycle fraction against 256 CUs x 4 SIMDs x 2.4 GHz."""
import csv
import json
import sys
from collections import defaultdict

SIMD_CYCLES_PER_S = 256 * 4 * 2.4e9


def bare(name):
    return name.split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]


def main(path, batch, rate=None, out=None):
    tot = defaultdict(lambda: defaultdict(float))
    loads = set()
    for r in csv.DictReader(open(path)):
        k = bare(r["Kernel_Name"])
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if k == "k_load_values":
            loads.add(r["Dispatch_Id"])
    nb = max(len(loads), 1)  # every batch launches k_load_values once
    rows = []
    for k, c in tot.items():
        if not k.startswith("k_"):
            continue
        insts = c.get("SQ_INSTS_VALU", 0) / nb / batch
        cyc = 4 * c.get("SQ_ACTIVE_INST_VALU", 0) / nb / batch
        i64 = c.get("SQ_INSTS_VALU_INT64", 0) / nb / batch
        i32 = c.get("SQ_INSTS_VALU_INT32", 0) / nb / batch
        rows.append((k, insts, cyc, i32, i64))
    rows.sort(key=lambda r: -r[2])
    ti = sum(r[1] for r in rows)
    tc = sum(r[2] for r in rows)
    print(f"{'kernel':20s} {'VALU inst/wit':>13s} {'VALU cyc/wit':>13s} {'cyc/inst':>8s} {'int32/wit':>10s} {'int64/wit':>10s}")
    for k, i, c, i32, i64 in rows:
        print(f"{k:20s} {i:13.0f} {c:13.0f} {c / i if i else 0:8.2f} {i32:10.0f} {i64:10.0f}")
    print(f"{'total':20s} {ti:13.0f} {tc:13.0f} {tc / ti if ti else 0:8.2f}")
    res = {"source": path, "batch": batch, "valu_insts_per_witness": round(ti, 1),
           "valu_cycles_per_witness": round(tc, 1),
           "kernels": {k: {"valu_insts_per_witness": round(i, 1), "valu_cycles_per_witness": round(c, 1),
                           "int32_per_witness": round(i32, 1), "int64_per_witness": round(i64, 1)}
                       for k, i, c, i32, i64 in rows}}
    if rate:
        res["witnesses_per_s"] = rate
        res["valu_cycle_frac"] = round(tc * rate / SIMD_CYCLES_PER_S, 3)
        res["valu_inst_frac"] = round(ti * rate / (SIMD_CYCLES_PER_S / 2), 3)
        print(f"at {rate:.0f} witnesses/s: VALU cycles {res['valu_cycle_frac']:.3f} of 256 x 4 SIMDs x 2.4 GHz "
              f"(instructions {res['valu_inst_frac']:.3f} of one per 2 cycles)")
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), float(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[3] != "-" else None,
         sys.argv[4] if len(sys.argv) > 4 else None)
