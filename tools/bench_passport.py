"""Host throughput of the bulk SOD preprocessor (pzk_passport_inputs): synthetic EF.SOD passports
(pzkwit.sodgen, canonical LDS layout) -> input rows, on 1 thread and on all of them.
    python tools/bench_passport.py [--n 8192] [--sig 1] [--ref /root/reference/test]
With --ref (this container only) it also times the reference's processPassport on Node over a sample
of the same files, as a per-passport CPU baseline for the step it replaces."""
import argparse
import base64
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "passport-zk-circuits_amd"))

from pzkwit import passport as PP, sodgen  # noqa: E402

NODE_TIMER = r"""
const path = require("path"), fs = require("fs"), os = require("os");
const { processPassport } = require(path.join(process.argv[2], "process_passport.js"));
const dir = process.argv[3], files = fs.readdirSync(dir).filter((f) => f.endsWith(".json")).sort();
const work = fs.mkdtempSync(path.join(os.tmpdir(), "ppb-"));
fs.mkdirSync(path.join(work, "test", "circuits", "generated"), { recursive: true });
fs.mkdirSync(path.join(work, "test", "inputs", "generated"), { recursive: true });
process.chdir(work);
const t0 = process.hrtime.bigint();
for (const f of files) processPassport(path.join(dir, f));
console.log(JSON.stringify({ n: files.length, s: Number(process.hrtime.bigint() - t0) / 1e9 }));
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--sig", type=int, default=1)
    ap.add_argument("--distinct", type=int, default=256, help="distinct passports (the batch repeats them)")
    ap.add_argument("--ref", default=None)
    ap.add_argument("--ref-sample", type=int, default=64)
    a = ap.parse_args()
    key = sodgen.signer_key(a.sig)
    uniq = [sodgen.make_passport(a.sig, key, i) for i in range(a.distinct)]
    batch = [uniq[i % len(uniq)] for i in range(a.n)]
    params = PP.parse(batch[0])["params"]
    res = {"sig": a.sig, "passports": a.n, "params": params, "threads": {}}
    rows, _ = PP.input_rows(params, batch[:1])
    rows = __import__("numpy").zeros((a.n,) + rows.shape[1:], dtype=rows.dtype)
    rows.fill(1)  # fault the pages in: the timed calls write rows into resident (e.g. pinned) memory
    srcs = PP.sources(batch)
    for th in (1, int(os.environ.get("OMP_NUM_THREADS", 0)) or len(os.sched_getaffinity(0))):  # the box's CPU share
        t = time.perf_counter()
        rows, st = PP.input_rows(params, srcs, threads=th, out=rows)
        dt = time.perf_counter() - t
        assert (st == 0).all()
        res["threads"][th] = {"s": dt, "passports_per_s": a.n / dt, "row_GB_per_s": rows.nbytes / dt / 1e9}
    if a.ref:
        with tempfile.TemporaryDirectory() as tmp:
            for i, pp in enumerate(uniq[:a.ref_sample]):
                with open(os.path.join(tmp, "p%05d.json" % i), "w") as fh:
                    json.dump({f: base64.b64encode(pp[f]).decode() for f in ("dg1", "dg15", "sod")}, fh)
            js = os.path.join(tmp, "timer.js")
            open(js, "w").write(NODE_TIMER)
            out = subprocess.check_output(["node", "--harmony-optional-chaining", "--harmony-private-methods", js,
                                           a.ref, tmp])
            r = json.loads(out.decode().strip().splitlines()[-1])
            res["reference_processPassport"] = {"passports": r["n"], "s": r["s"], "passports_per_s": r["n"] / r["s"],
                                                "threads": 1, "runtime": "node " + subprocess.check_output(
                                                    ["node", "--version"]).decode().strip()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
