#!/usr/bin/env python3
"""bench.py — RegisterIdentityBuilder witnesses/s on MI355X (BASELINE.json metric).

python bench.py --gpus N --steps K --warmup W [--workload register|sha256]

One step = one pass of the hot path over one batch of synthetic passports per GPU
(batch 4096 of the canonical instance RegisterIdentityBuilder(1,256,3,4,600,248,1,1496,3,256),
SURVEY.md §8d config 3), inputs already resident in HBM when the timed region starts.
A full --O0 witness is ~72 MB, so a 4096 batch (~295 GB) does not fit one GPU's 288 GB:
each step runs it as sub-batches into a reused output slab (every witness is fully
written). N > 1 shards the batch (weak scaling, no data-path collective).
Rank 0 prints ONE JSON line.
"""
import argparse
import glob
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "passport-zk-circuits_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles per SIMD (MI355X_MICROARCH.md: a wave
# issues each VALU instruction over 2 cycles), 2.4 GHz max clock -> G wave-instructions/s
VALU_PEAK_GIPS = 256 * 4 * 2.4 / 2
# Measured chip-wide issue rates (tools/fieldbench/issuebench.hip, profiles/r6p/issuebench.txt; 8 waves per SIMD,
# independent chains): v_add_u32 975 G wave-instr/s; v_mad_u64_u32 515, v_lshl_add_u64 518, v_add_co_u32 541,
# v_mul_lo_u32 549, v_mul_hi_u32 570, DPP moves 584. The field arithmetic is mostly of the second kind.
VALU_RATE_SIMPLE_GIPS = 975.0
VALU_RATE_INT64_GIPS = 515.0
VALU_RATE_CARRY_GIPS = 541.0


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


# ----------------------------------------------------------------------------- inputs
def smt_depth_of(spec, i):
    """SMT proof depth of passport i: spec "0" (the default: a one-leaf registration tree, every level below the
    insertion level hashes Poseidon(0, 0)) or "A-B" (uniform over A..B by a hash of i, e.g. 20-30 for a tree of
    about a million identities, 40-79 for config 4's deep proofs)."""
    if "-" not in str(spec):
        return int(spec)
    a, b = (int(x) for x in str(spec).split("-"))
    return a + ((i * 0x9E3779B1) >> 7) % (b - a + 1)


def _gen_slice(args):
    seed, lo, hi, n_keys, sig = args[:5]
    depth = args[5] if len(args) > 5 else "0"
    root = args[6] if len(args) > 6 else False
    from pzkwit import inputs as I
    g = I.PassportGen.shared(seed, n_keys, sig)
    out = np.zeros((hi - lo, g.n_inputs, 32), dtype=np.uint8)
    for k, i in enumerate(range(lo, hi)):
        I.pack_register_inputs(g.passport_at(i, smt_depth=smt_depth_of(depth, i), smt_root=root), g.params, out=out[k])
    return lo, out


def make_register_inputs(batch, first, seed=3, n_keys=64, workers=None, sig=1, smt_depth="0", smt_root=False):
    """Passports first .. first + batch - 1 of the synthetic stream, packed. smt_root: with deep
    proofs, slaveMerkleRoot = the proof's root (Python Poseidon; config 4) instead of 0."""
    from pzkwit import inputs as I
    workers = workers or max(1, min(16, os.cpu_count() or 1))
    keys = I.PassportGen.shared(seed, n_keys, sig).keys  # keys generated once (parallel inside), handed to workers
    step = (batch + workers * 4 - 1) // (workers * 4)
    jobs = [(seed, first + lo, first + min(batch, lo + step), n_keys, sig, smt_depth, smt_root)
            for lo in range(0, batch, step)]
    n_in = I.PassportGen.shared(seed, n_keys, sig).n_inputs
    buf = np.zeros((batch, n_in, 32), dtype=np.uint8)
    if workers == 1:
        for lo, arr in map(_gen_slice, jobs):
            buf[lo - first: lo - first + len(arr)] = arr
    else:
        with I.process_pool(workers, I.PassportGen.install_shared, (seed, n_keys, sig, keys)) as ex:
            for lo, arr in ex.map(_gen_slice, jobs):
                buf[lo - first: lo - first + len(arr)] = arr
    return buf


# ----------------------------------------------------------------------------- CPU baseline
# workload -> SIGNATURE_TYPE of the RegisterIdentityBuilder instance, and its input seed
WL_SIG = {"register": 1, "register-ecdsa": 20, "register-pss": 11, "register-brainpool": 21, "config4": 1}
SIG_SEED = {1: 3, 2: 4, 3: 11, 4: 12, 10: 6, 11: 7, 12: 8, 13: 13, 14: 10, 20: 5, 21: 9, 24: 14, 25: 15}
CPU_SHARE = 16  # host CPUs a one-GPU job may use on the GPU box (its OMP_NUM_THREADS / MAX_JOBS)
# the canonical instance, seed 0x4, SMT proofs of depth uniform in 1..79 (non-zero siblings
# below the depth, zeros above), slaveMerkleRoot = the proof's root
CONFIG4 = {"seed": 4, "smt_depth": "1-79"}
CONFIG4_WORKLOAD = ("RegisterIdentityBuilder(1,256,3,4,600,248,1,1496,3,256) synthetic passports, SMT proofs of depth "
                    "1-79 (config 4, seed 0x4)")
# PoseidonHash(2) of the KATs (0,0), (1,2), (p-1,p-1) and 1,000 pairs from SplitMix64 seed 0x1
POSEIDON_BATCH = 1 << 20


def register_like(workload):
    return workload.startswith("register") or workload == "config4"


def workload_seed(args):
    return CONFIG4["seed"] if args.workload == "config4" else SIG_SEED[args.sig_eff]


def workload_depth(args):
    depth = getattr(args, "smt_depth", "0")
    if args.workload == "config4" and depth == "0":
        return CONFIG4["smt_depth"]
    return depth


def poseidon_config1_pairs():
    """Config 1's 1,003 input pairs (the order of tools/gen_poseidon_kats.js)."""
    from pzkwit import field
    pairs = [(0, 0), (1, 2), (field.P - 1, field.P - 1)]
    rng = field.SplitMix64(1)
    pairs += [(rng.fr(), rng.fr()) for _ in range(1000)]
    return pairs


def poseidon_rows(n):
    """n input rows of PoseidonHash(2): config 1's pairs, repeated. -> (n, 2, 32) uint8"""
    pairs = poseidon_config1_pairs()
    uniq = np.zeros((len(pairs), 2, 32), dtype=np.uint8)
    for i, (a, b) in enumerate(pairs):
        uniq[i, 0] = np.frombuffer(a.to_bytes(32, "little"), dtype=np.uint8)
        uniq[i, 1] = np.frombuffer(b.to_bytes(32, "little"), dtype=np.uint8)
    return uniq[np.arange(n) % len(pairs)]


def _cpu_work(args):
    kind, rows = args
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    from pzkwit import inputs as I
    if kind.startswith("register"):
        prm = pyoracle.register_params(**I.instance_params(int(kind.split(":")[1])))
        nin, nw = pyoracle.register_sizes(prm)
        w = np.zeros((nw, 32), dtype=np.uint8)
        for r in rows:
            pyoracle.register_witness(prm, r, out=w)
    elif kind == "poseidon":
        for r in rows:
            rc, _ = pyoracle.poseidon_witness([int.from_bytes(bytes(e), "little") for e in r])
            assert rc == 0
    elif kind.startswith("query"):
        td1 = kind == "query-td1"
        w = np.zeros((pyoracle.query_sizes(td1)[1], 32), dtype=np.uint8)
        for r in rows:
            pyoracle.query_witness(r, out=w, td1=td1)
    else:
        for r in rows:
            pyoracle.sha256_witness(r, 6)
    return len(rows)


def cpu_baseline(kind, sample_rows, procs):
    """The CPU restatement (oracle/, kind "port") on a bounded sample, one witness per process."""
    from pzkwit import inputs as I
    chunks = [(kind, sample_rows[i::procs]) for i in range(procs)]
    with I.process_pool(procs) as ex:
        list(ex.map(_cpu_work, [(kind, sample_rows[:1])] * procs))  # warm (lib load)
        t0 = time.perf_counter()
        n = sum(ex.map(_cpu_work, chunks))
        dt = time.perf_counter() - t0
    return n / dt, dt


def cpu_baseline_1thread(kind, sample_rows):
    _cpu_work((kind, sample_rows[:1]))  # warm
    t0 = time.perf_counter()
    n = _cpu_work((kind, sample_rows))
    dt = time.perf_counter() - t0
    return n / dt, dt


# ----------------------------------------------------------------------------- ranks
def launch_ranks(n):
    """--gpus N without a launcher: start N ranks (one process per GPU) through
    torch.distributed.run as a child process and exit with its code. Runs before anything
    imports torch or touches the GPU."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % n,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + sys.argv[1:]
    log("launching %d ranks: %s" % (n, " ".join(cmd)))
    return subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))


class GpuEngine:
    """The measured path: libpzkwit on cuda:local, sub-batches written into a ring of output slots.

    Calls go to the instance's own streams (pipelined: sub-batch k + 1's cores run beside
    sub-batch k's emitters); the step ends with a device synchronise."""

    def __init__(self, args, workload, dev):
        import torch
        from pzkwit import native, inputs as I
        self.torch, self.dev = torch, dev
        self.layout = "O0 (all signals)"
        self.layout_key = args.sym if getattr(args, "sym", None) else "O0"  # PMC pass lookup (pmc_pass)
        if register_like(workload) or workload.startswith("query"):
            if register_like(workload):
                circuit, size_arg, params = native.PZK_CIRCUIT_REGISTER, 0, I.instance_params(args.sig_eff)
                n_in = I.PassportGen.shared(workload_seed(args), 64, args.sig_eff).n_inputs
                shape = {1: "register_canonical", 20: "register_sig20"}.get(args.sig_eff)
            else:
                circuit, size_arg, params = native.PZK_CIRCUIT_QUERY, 80, {"doc": 1 if workload == "query-td1" else 0}
                n_in = native.layout_info(params, circuit, size_arg).n_inputs
                shape = "query" if workload == "query" else None
            n_o0 = native.layout_info(params, circuit, size_arg).witness_size
            sym = None
            if getattr(args, "sym", None):
                from pzkwit import symmap
                if args.sym.startswith("synthetic"):
                    frac = int(args.sym.split(":")[1]) if ":" in args.sym else 4
                    keep = symmap.synthetic_keep(n_o0, 1 + 4 + n_in, fraction=frac)
                    sym = symmap.sym_text(keep)
                    self.layout = ("synthetic .sym map: outputs + inputs + 1/%d of the O0 signals (hash subset; NOT "
                                   "circom's O2, which cannot be built here)" % frac)
                elif args.sym in ("o1shape", "o2shape"):
                    level = int(args.sym[1])
                    if shape is None:
                        raise SystemExit("--sym %s: no committed shape map for this workload (tools/gen_shape_maps.py)"
                                         % args.sym)
                    wit = symmap.load_shape(shape, level)
                    sym = symmap.sym_text_wit(wit)
                    self.layout = ("circom --O%d-shaped .sym map (data/shape/%s_o%d.npz: circom's documented "
                                   "simplification applied to the restated constraints, %d of %d signals; which "
                                   "signals circom itself keeps is parity unpinned)"
                                   % (level, shape, level, int(wit.max()), n_o0 - 1))
                else:
                    sym = open(args.sym).read()
                    self.layout = ".sym map %s" % os.path.basename(args.sym)
            self.inst = native.Instance(circuit, size_arg, params, sym=sym)
            if sym is not None:
                inv = symmap.parse_sym(sym)
                if (np.diff(inv) <= 0).any() or os.environ.get("PZK_SYM_GATHER"):  # two O0 staging chunks of <= 1024 witnesses
                    self.o0_staging_bytes = 2 * 1024 * 32 * n_o0
                    self.layout += "; staging + gather (non-monotone map)"
                else:
                    self.layout += "; emitted directly (monotone map, mapsink.hpp)"
            if workload.startswith("query"):
                self.layout += ("; BabyPbk (identityStateVerifier.circom:19, undefined in the snapshot) substituted by "
                                "the reference's BabyjubjubBase8Multiplication (DESIGN.md §11)")
        elif workload == "poseidon":
            self.inst = native.Instance(native.PZK_CIRCUIT_POSEIDON, 2)
        else:
            self.inst = native.Instance(native.PZK_CIRCUIT_SHA256, 6)
        self.W, self.NIN = self.inst.witness_size, self.inst.n_inputs
        self.n_pub = self.inst.n_outputs + self.inst.n_public_inputs

    def setup(self, d_in, batch, sub, slots, steps):
        torch = self.torch
        self.d_in, self.batch, self.sub, self.slots = d_in, batch, sub, slots
        self.stride = 32 * self.W
        self.d_out = torch.empty(slots * sub * self.stride, dtype=torch.uint8, device=self.dev)
        self.d_st = torch.zeros((max(steps, 1), batch), dtype=torch.int32, device=self.dev)
        torch.cuda.synchronize(self.dev)  # inputs / buffers made on torch's stream: the library's streams do not wait for it

    def step(self, k, timing):
        for j, lo in enumerate(range(0, self.batch, self.sub)):
            n = min(self.sub, self.batch - lo)
            slot = j % self.slots
            self.inst.witness_batch_device(self.d_in.data_ptr() + lo * self.NIN * 32, n,
                                           self.d_out.data_ptr() + slot * self.sub * self.stride, self.stride,
                                           self.d_st[k].data_ptr() + 4 * lo, timing=timing)

    def sync(self):
        self.inst.sync()
        self.torch.cuda.synchronize(self.dev)

    def statuses(self, steps):
        return self.d_st[:steps]

    def public_pass(self):
        """Untimed pass after the timed region: status and public signals (witness[1 ..]) of every
        witness of the batch, for the gather."""
        torch = self.torch
        st = torch.zeros(self.batch, dtype=torch.int32, device=self.dev)
        pub = torch.zeros((self.batch, self.n_pub, 32), dtype=torch.uint8, device=self.dev)
        out = self.d_out[: self.sub * self.stride].view(self.sub, self.W, 32)
        for lo in range(0, self.batch, self.sub):
            n = min(self.sub, self.batch - lo)
            self.inst.witness_batch_device(self.d_in.data_ptr() + lo * self.NIN * 32, n, self.d_out.data_ptr(),
                                           self.stride, st.data_ptr() + 4 * lo)
            self.inst.sync()
            pub[lo: lo + n] = out[:n, 1: 1 + self.n_pub]
        torch.cuda.synchronize(self.dev)
        return st, pub


def host_rows(args, workload, n, world):
    """Rank 0: the whole job's input rows of a workload on the host. -> (n, NIN, 32) uint8"""
    from pzkwit import inputs as I
    workers = max(1, min(CPU_SHARE * world, os.cpu_count() or 1))
    if workload == "config4":
        return make_register_inputs(n, 0, seed=CONFIG4["seed"], sig=1, workers=workers, smt_depth=CONFIG4["smt_depth"],
                                    smt_root=True)
    if register_like(workload):
        return make_register_inputs(n, 0, seed=workload_seed(args), sig=args.sig_eff, workers=workers,
                                    smt_depth=workload_depth(args), smt_root=args.workload == "config4")
    if workload.startswith("query"):
        from pzkwit import query as Q
        return Q.batch_rows(n, seed=0x9, distinct=64, td1=workload == "query-td1")
    if workload == "poseidon":
        return poseidon_rows(n)
    _, host = I.sha256_config2_batch(n, seed=2, blocks=6)
    return host


def scatter_rows(d_in, full, dist, dev):
    """Shard r of the job's rows (rank 0's host tensor [world, shard bytes]) into rank r's device buffer."""
    if dist is None:
        d_in.copy_(full[0])
    else:
        parts = list(full.to(dev).unbind(0)) if full is not None else None
        dist.scatter(d_in, parts, src=0)
        del parts


def timed_steps(engine, args, dist):
    """W untimed warmup steps, then exactly K timed steps between barriers + device synchronisation.
    -> (seconds, lanes failing in the timed steps)"""
    for _ in range(args.warmup):
        engine.step(0, False)
    engine.sync()
    if hasattr(engine.inst, "timing"):
        engine.inst.timing(reset=True)
    if dist:
        dist.barrier()
    engine.sync()
    t0 = time.perf_counter()
    for k in range(args.steps):
        engine.step(k, True)
    engine.sync()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    bad = int((engine.statuses(args.steps) != 0).sum().item())
    return dt, bad


def reduce_run(dist, dev, dt, bad):
    """max of the timed seconds and sum of the failing lanes over ranks"""
    if not dist:
        return dt, bad
    import torch
    tt = torch.tensor([dt], device=dev, dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    bt = torch.tensor([bad], device=dev, dtype=torch.int64)
    dist.all_reduce(bt)
    return float(tt.item()), int(bt.item())


def wants_config4(args):
    """The default register line also measures config 4 on the same instance, reported beside the
    headline config-3 value (`config4` key); with --sym on the mapped instance (the prover-facing layout with real
    SMT proofs)."""
    return (args.workload == "register" and args.sig_eff == 1 and getattr(args, "smt_depth", "0") == "0"
            and not getattr(args, "no_config4", False))


def run_rank(args, rank, world, local, dist, engine_cls=GpuEngine, device="cuda"):
    """One rank of the bench (also driven by tests/test_host.py over gloo with a stub engine).

    Rank 0 generates the whole job's inputs on the host, ranks receive their contiguous shard from
    it over the process group (RCCL point-to-point scatter on GPUs), run W + K steps, and the
    per-lane status + public signals are all-gathered after the timed region. The default register line then
    runs config 4's inputs through the same instance the same way. Returns the record for rank 0's report."""
    import torch
    from pzkwit import dist as D
    dev = torch.device(device, local) if device == "cuda" else torch.device(device)
    register = register_like(args.workload)
    batch = args.batch or (4096 if register or args.workload.startswith("query")
                           else POSEIDON_BATCH if args.workload == "poseidon" else 1024)
    engine = engine_cls(args, args.workload, dev)
    NIN, W = engine.NIN, engine.W
    # inputs: rank 0 makes all world x batch rows, scatters shard r to rank r
    t0 = time.time()
    full = None
    if rank == 0:
        full = torch.from_numpy(host_rows(args, args.workload, batch * world, world).reshape(world, -1))
        log("inputs: %d x %d rows generated on rank 0 in %.1fs" % (world, batch, time.time() - t0))
    d_in = torch.empty(batch * NIN * 32, dtype=torch.uint8, device=dev)
    scatter_rows(d_in, full, dist, dev)
    del full

    stride = 32 * W
    # ring of output slots. With one slot, consecutive sub-batches still overlap safely: each emitter
    # kind runs on one fixed stream, so a region of a row is rewritten only after the previous
    # sub-batch's write of that region
    slots = args.slots
    if args.sub:
        sub = min(args.sub, batch)
    elif device == "cuda":
        free, _ = torch.cuda.mem_get_info(dev)
        # per-witness core scratch (EC value tables dominate: 11 / 15 / 20 MB for P-256 / P-224 / brainpoolP384r1), two sets
        scratch_pw = {24: 16 << 20, 25: 22 << 20}.get(args.sig_eff, 10 << 20 if args.sig_eff >= 20 else 1 << 20)
        staging = getattr(engine, "o0_staging_bytes", 0)  # mapped layouts: the library's O0 chunk slots
        fit = max(1, int((free * 0.85 - staging) // (slots * stride + 2 * scratch_pw)))
        parts_n = 1
        while (batch + parts_n - 1) // parts_n > fit:
            parts_n += 1
        sub = (batch + parts_n - 1) // parts_n
    else:
        sub = batch
    sub = min(sub, 32768)  # pzk_witness_batch takes <= 65535 witnesses per call (its grids' y dimension)
    slots = min(slots, (batch + sub - 1) // sub)
    log("witness_size=%d (%.1f MB), batch=%d, sub-batch=%d, %d output slots %.1f GB" % (
        W, stride / 1e6, batch, sub, slots, slots * sub * stride / 1e9))
    engine.setup(d_in, batch, sub, slots, args.steps)

    dt, bad = timed_steps(engine, args, dist)
    timing = engine.inst.timing() if hasattr(engine.inst, "timing") else None
    st, pub = engine.public_pass()
    dt, bad = reduce_run(dist, dev, dt, bad)
    if dist:
        st, pub = D.gather_results(dist, st, pub, device=dev)
    import hashlib
    gathered = {"witnesses": int(st.shape[0]), "status_nonzero": int((st != 0).sum().item()),
                "public_signals": int(pub.shape[1]),
                "public_sha256": hashlib.sha256(pub.cpu().numpy().tobytes()).hexdigest()[:16]}
    c4 = None
    if wants_config4(args):
        t0 = time.time()
        full = None
        if rank == 0:
            full = torch.from_numpy(host_rows(args, "config4", batch * world, world).reshape(world, -1))
            log("config 4 inputs: %d x %d rows generated on rank 0 in %.1fs" % (world, batch, time.time() - t0))
        scatter_rows(d_in, full, dist, dev)
        del full
        engine.sync()
        d4, b4 = reduce_run(dist, dev, *timed_steps(engine, args, dist))
        t4 = engine.inst.timing() if hasattr(engine.inst, "timing") else None
        c4 = dict(dt=d4, bad=b4, timing=t4)
    return dict(dt=dt, bad=bad, batch=batch, sub=sub, slots=slots, W=W, NIN=NIN, engine=engine,
                gathered=gathered, timing=timing, config4=c4)


# ----------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=["register", "register-ecdsa", "register-pss", "register-brainpool", "config4",
                                           "sha256", "poseidon", "mixed", "query", "query-td1"], default="register")
    ap.add_argument("--sig", type=int, default=None, help="SIGNATURE_TYPE of a register workload (overrides --workload's)")
    ap.add_argument("--batch", type=int, default=None, help="witnesses per GPU per step")
    ap.add_argument("--sub", type=int, default=None, help="sub-batch (output slot) size")
    ap.add_argument("--slots", type=int, default=1, help="output slots (ring) per GPU")
    ap.add_argument("--sym", default=None, help="signal -> witness map: a circom .sym file, o1shape / o2shape (the "
                    "committed circom-shaped maps), or synthetic[:N]")
    ap.add_argument("--smt-depth", default="0", help="register workloads: SMT proof depth of the synthetic "
                    "passports, N or A-B (uniform); default 0 (a one-leaf registration tree)")
    ap.add_argument("--no-config4", action="store_true", help="default register line: skip the embedded config-4 "
                    "measurement")
    ap.add_argument("--cpu-sample", type=int, default=None)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host", action="store_true", help="skip the host_delivered (streamed) measurement")
    ap.add_argument("--host-sample", type=int, default=None, help="witnesses streamed for host_delivered")
    args = ap.parse_args()
    if args.workload == "mixed" and os.environ.get("PZK_MIX_HWQ", "keep") != "keep":
        # PZK_MIX_HWQ=N (A/B): GPU_MAX_HW_QUEUES for the mixed line, set before any HIP call and inherited by the ranks
        # launch_ranks starts. Default: the environment's value (the boxes' 4). Round 4 needed 16 (40.9k -> 43.2k
        # witnesses/s, profiles/r4_hwq/); since the instances sharing a device take the reduced stream set
        # (runtime.cpp ensure_chain_streams) the line holds at 4: 46.9k (profiles/r6i/)
        hwq = os.environ.get("PZK_MIX_HWQ")
        if not hwq.isdigit() or not 1 <= int(hwq) <= 32:
            raise SystemExit("PZK_MIX_HWQ=%s: expected an integer 1..32 (hardware queues per process) or 'keep'" % hwq)
        if os.environ.get("GPU_MAX_HW_QUEUES") != hwq:
            log("mixed workload: GPU_MAX_HW_QUEUES %s -> %s (PZK_MIX_HWQ; 'keep' leaves it)"
                % (os.environ.get("GPU_MAX_HW_QUEUES", "unset"), hwq))
        os.environ["GPU_MAX_HW_QUEUES"] = hwq
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args.gpus)  # before torch / any GPU call
    args.sig_eff = (args.sig or WL_SIG[args.workload]) if register_like(args.workload) else 0
    if args.workload == "config4" and args.sig not in (None, 1):
        raise SystemExit("--workload config4 is SIGNATURE_TYPE 1 (SURVEY.md §8d)")
    if args.workload == "mixed":
        return bench_mixed(args)

    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        log("note: WORLD_SIZE=%d ranks (launcher) for --gpus %d" % (world, args.gpus))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    r = run_rank(args, rank, world, local, dist)
    if rank == 0:
        print(json.dumps(report(args, r, world)), flush=True)
    if dist:
        dist.destroy_process_group()


def workload_name(args):
    """(metric, config.workload) of the line"""
    from pzkwit import inputs as I
    sig = args.sig_eff
    if args.workload == "config4":
        return "registerIdentityBuilder witnesses/sec, batch=4096, 1 & 8 MI355X; % HBM roofline", CONFIG4_WORKLOAD
    if args.workload.startswith("register"):
        metric = "registerIdentityBuilder witnesses/sec, batch=4096, 1 & 8 MI355X; % HBM roofline"
        workload = "RegisterIdentityBuilder(1,256,3,4,600,248,1,1496,3,256) synthetic passports (config 3)"
        if sig == 21:
            metric = "registerIdentityBuilder ECDSA-brainpoolP256r1 witnesses/sec, batch=4096 (SIGNATURE_TYPE 21)"
            workload = "RegisterIdentityBuilder(21,256,3,4,600,248,1,1496,3,256) synthetic brainpoolP256r1 passports"
        elif sig == 20:
            metric = "registerIdentityBuilder ECDSA-secp256r1 witnesses/sec, batch=4096 (config 5 slice)"
            workload = "RegisterIdentityBuilder(20,256,3,4,600,248,1,1496,3,256) synthetic P-256 passports"
        elif sig == 11:
            metric = "registerIdentityBuilder RSA-PSS witnesses/sec, batch=4096 (SIGNATURE_TYPE 11)"
            workload = "RegisterIdentityBuilder(11,256,3,4,600,248,1,1496,3,256) synthetic RSA-2048 PSS passports"
        elif sig != 1:
            metric = "registerIdentityBuilder witnesses/sec, batch=4096 (SIGNATURE_TYPE %d)" % sig
            q = I.instance_params(sig)
            workload = "RegisterIdentityBuilder(%d,%d,%d,%d,%d,%d,%d,%d,%d,%d) synthetic passports" % tuple(
                q[k] for k in ("sig", "dg_hash", "doc", "ec_blocks", "ec_shift", "dg1_shift", "aa", "dg15_shift",
                               "dg15_blocks", "aa_shift"))
        if getattr(args, "smt_depth", "0") != "0":
            workload = workload.replace(" (config 3)", "") + ", SMT proofs of depth %s" % args.smt_depth
        return metric, workload
    if args.workload.startswith("query"):
        td1 = args.workload == "query-td1"
        return ("QueryIdentity%s(80) witnesses/sec, batch=4096 (SURVEY.md row f4)" % ("TD1" if td1 else ""),
                "QueryIdentity%s(80) synthetic queries (64 distinct, SMT proofs of depth 0-79)" % ("TD1" if td1 else ""))
    if args.workload == "poseidon":
        return ("PoseidonHash(2) witnesses/sec (config 1)",
                "PoseidonHash(2) of config 1's 1,003 input pairs (KATs (0,0), (1,2), (p-1,p-1) + 1,000 SplitMix64 "
                "seed 0x1 pairs), repeated to the batch")
    return ("Sha256HashChunks(6) witnesses/sec, batch=1024 (config 2)",
            "Sha256HashChunks(6) synthetic 312-375 B messages (config 2)")


def pmc_pass(workload, layout_key):
    """The committed PMC pass of a workload + layout (profiles/pmc_*/traffic.json, tools/pmc_summary.py): the last
    one in name order, or None"""
    found = None
    for tf in sorted(glob.glob(os.path.join(REPO, "profiles", "pmc_*", "traffic.json"))):
        tj = json.load(open(tf))
        if tj.get("workload") == workload and tj.get("layout_key", "O0") == layout_key:
            found = (tf, tj)
    return found


def valu_roofline(tj, tf, value, world):
    """whole-job VALU roofline: wave-level VALU instructions per witness (SQ_INSTS_VALU summed over the job's
    kernels, from the committed PMC pass of this workload) x witnesses/s against the chip's VALU issue rate"""
    if not tj or not tj.get("valu_insts_per_witness"):
        return None
    ipw = tj["valu_insts_per_witness"]
    ach = ipw * value / 1e9
    top = sorted(((v.get("valu_insts_per_witness", 0), k) for k, v in tj["kernels"].items()), reverse=True)[:3]
    res = {"bound": "valu", "insts_per_witness": ipw, "achieved": round(ach, 1), "peak": VALU_PEAK_GIPS,
           "unit": "G wave-instr/s", "frac": round(ach / (VALU_PEAK_GIPS * world), 4),
           "top_kernels": {k: v for v, k in top}, "source": os.path.relpath(tf, REPO),
           "note": "issue-rate bound (1 wave64 VALU instruction / 2 cycles / SIMD at 2.4 GHz); 64-bit "
                   "integer multiply-adds take more than one issue slot, so the attainable fraction is < 1"}
    # the instruction classes of the same workload (tools/pmc_valu.py: SQ_INSTS_VALU_INT64 beside SQ_INSTS_VALU), priced
    # at the measured issue rates: INT64 at v_mad_u64_u32's, the rest between v_add_u32's (lo) and a carry add's (hi)
    vf = os.path.join(os.path.dirname(tf), "valu.json")
    if os.path.exists(vf):
        vj = json.load(open(vf))
        i64 = sum(k.get("int64_per_witness", 0) for k in vj["kernels"].values())
        rest = max(vj["valu_insts_per_witness"] - i64, 0.0)
        busy = lambda r: value / world * (i64 / (VALU_RATE_INT64_GIPS * 1e9) + rest / (r * 1e9))
        res["measured_issue"] = {"int64_per_witness": round(i64, 1), "other_per_witness": round(rest, 1),
                                 "frac_lo": round(busy(VALU_RATE_SIMPLE_GIPS), 4),
                                 "frac_hi": round(busy(VALU_RATE_CARRY_GIPS), 4),
                                 "rates_gips": {"int64": VALU_RATE_INT64_GIPS, "simple": VALU_RATE_SIMPLE_GIPS,
                                                "carry": VALU_RATE_CARRY_GIPS},
                                 "source": os.path.relpath(vf, REPO)}
    return res


def phase_table(tm, info):
    return {p: {"ms_per_launch": round(tm[p][0] / max(tm[p][1], 1), 4), "launches": tm[p][1],
                "kernel": info[p][0], "alg_bytes_per_witness": info[p][1]} for p in tm if tm[p][1]}


def report(args, r, world):
    from pzkwit import inputs as I
    sig = args.sig_eff
    metric, workload = workload_name(args)
    dt, batch, sub, W, NIN, inst = r["dt"], r["batch"], r["sub"], r["W"], r["NIN"], r["engine"].inst
    value = batch * world * args.steps / dt
    layout_key = getattr(r["engine"], "layout_key", "O0")

    # roofline of the dominant kernel (HIP events on the launch stream, inside the timed region)
    tm = r.get("timing") or inst.timing()
    info = {n: (k, b) for n, k, b in inst.phase_info()}
    # the dominant kernel = the one carrying the most algorithmic bytes (k_emit_sha: ~75 % of the witness)
    dom = max((p for p in tm if tm[p][1] > 0), key=lambda p: info[p][1])
    ms_total, launches = tm[dom]
    avg_ms = ms_total / launches
    # launches cover ragged sub-batches: bytes per launch = bytes of all timed witnesses / launches
    bytes_per_launch = info[dom][1] * batch * args.steps / launches
    achieved = bytes_per_launch / (avg_ms / 1e3) / 1e9
    # PMC traffic (FETCH_SIZE x 2 + WRITE_SIZE per witness, tools/pmc_summary.py) from the committed pass of the
    # workload and layout this line measures; none -> null
    traffic, traffic_src = None, None
    pm = pmc_pass(workload, layout_key)
    tf, tj = pm if pm else (None, None)
    if tj:
        ks = [tj["kernels"].get(k) for k in info[dom][0].split("+")]
        if all(ks):
            traffic = sum(k["traffic_bytes_per_witness"] for k in ks) * batch * args.steps / launches
            traffic_src = os.path.relpath(tf, REPO)
    # whole-job algorithmic bytes: inputs read once + .wtns header and elements written once
    job_bytes = 32 * NIN + 76 + 32 * W
    job_gbs = value * job_bytes / 1e9
    valu = valu_roofline(tj, tf, value, world)
    # the same kernel alone (the PMC pass serialises dispatches): its bytes over its standalone time, for the share of
    # the concurrent schedule's HBM the other emitters take while it runs
    standalone = None
    if tj and all(tj["kernels"].get(k, {}).get("standalone_ms_per_batch") for k in info[dom][0].split("+")):
        sms = sum(tj["kernels"][k]["standalone_ms_per_batch"] for k in info[dom][0].split("+"))
        sb = info[dom][1] * tj["batch"]
        standalone = {"ms_per_launch": sms, "witnesses_per_launch": tj["batch"],
                      "achieved": round(sb / (sms / 1e3) / 1e9, 1), "frac": round(sb / (sms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                      "source": os.path.relpath(tf, REPO)}
    out = {
        "metric": metric, "value": round(value, 2), "unit": "witnesses/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "bn254_fr (u32 limbs)",
        "data": "synthetic",
        "config": {"workload": workload, "batch_per_gpu": batch, "sub_batch": sub, "output_slots": r["slots"],
                   "output": "device-resident generation: each sub-batch's .wtns rows are written to HBM into a "
                             "ring of output slots that the next sub-batches overwrite (a 4096 batch of 72 MB "
                             "witnesses exceeds one GPU's HBM); host delivery is not in the timed region",
                   "witness_elements": W, "witness_bytes": 32 * W, "layout": r["engine"].layout,
                   "layout_key": layout_key,
                   "smt_depth": workload_depth(args) if register_like(args.workload) else None,
                   "parallelism": "shard%d" % world, "invalid_lanes": r["bad"], "gathered": r["gathered"]},
        "roofline": {"bound": "hbm", "kernel": info[dom][0], "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_source": traffic_src, "bytes_per_launch": int(bytes_per_launch),
                     "avg_launch_ms": round(avg_ms, 4), "standalone": standalone, "valu": valu,
                     "job_bound": ("valu" if valu and valu["frac"] > job_gbs / (HBM_PEAK_GBS * world) else "hbm")},
        "job_hbm": {"alg_bytes_per_witness": job_bytes, "achieved": round(job_gbs, 1), "unit": "GB/s",
                    "frac": round(job_gbs / (HBM_PEAK_GBS * world), 4)},
        "phases": phase_table(tm, info),
    }
    c4 = r.get("config4")
    if c4:
        v4 = batch * world * args.steps / c4["dt"]
        g4 = v4 * job_bytes / 1e9
        pm4 = pmc_pass(CONFIG4_WORKLOAD, layout_key)
        out["config4"] = {
            "what": "SURVEY.md §8d config 4 on the same instance and sub-batching, measured after the headline line "
                    "(W warmup + K timed steps of its own inputs; the driver's 8-GPU run shards it 8 x %d)" % batch,
            "workload": CONFIG4_WORKLOAD, "value": round(v4, 2), "unit": "witnesses/s", "n_gpus": world,
            "ms_per_step": round(c4["dt"] / args.steps * 1e3, 3), "smt_depth": CONFIG4["smt_depth"],
            "seed": "0x%x" % CONFIG4["seed"], "slave_merkle_root": "the proof's root (Python Poseidon)",
            "invalid_lanes": c4["bad"],
            "job_hbm": {"achieved": round(g4, 1), "unit": "GB/s", "frac": round(g4 / (HBM_PEAK_GBS * world), 4)},
            "valu": valu_roofline(pm4[1], pm4[0], v4, world) if pm4 else None,
            "phases": phase_table(c4["timing"], info) if c4.get("timing") else None}
    if world == 1 and not args.no_host and register_like(args.workload):
        out["host_delivered"] = host_delivered(args, r["engine"].inst, sig)
    if world == 1 and not args.no_cpu and register_like(args.workload) and sig in (1, 3, 10, 11, 12, 20, 21, 24, 25):
        out["input_side"] = input_side(sig)
    if world == 1 and not args.no_cpu:  # CPU baseline: N = 1 only (bounded sample)
        procs = max(1, min(CPU_SHARE, os.cpu_count() or 1))
        if register_like(args.workload):
            ns = args.cpu_sample or (48 if sig >= 20 else 96 if sig == 11 else 128) * procs
            rows = make_register_inputs(ns, 10 ** 6, workers=procs, seed=workload_seed(args), sig=sig,
                                        smt_depth=workload_depth(args))
            kind = "register:%d" % sig
        elif args.workload.startswith("query"):
            from pzkwit import query as Q
            ns = args.cpu_sample or 64 * procs
            rows = Q.batch_rows(ns, seed=99, distinct=64, td1=args.workload == "query-td1")
            kind = args.workload
        elif args.workload == "poseidon":
            ns = args.cpu_sample or 1003 * 100 * procs  # ~10 s at the oracle's ~11k witnesses/s per process
            rows = poseidon_rows(ns)
            kind = "poseidon"
        else:
            ns = args.cpu_sample or 64 * procs
            _, rows = I.sha256_config2_batch(ns, seed=99, blocks=6)
            kind = args.workload
        rows = np.asarray(rows)  # slices of one array go to the worker processes (not a list of small arrays)
        v, cdt = cpu_baseline(kind, rows, procs)
        n1 = max(2, ns // (4 * procs))
        v1, cdt1 = cpu_baseline_1thread(kind, rows[:n1])
        try:
            affinity = len(os.sched_getaffinity(0))
        except AttributeError:
            affinity = os.cpu_count()
        nproc = os.cpu_count() or 1
        out["cpu_baseline"] = {
            "value": round(v, 2), "unit": "witnesses/s", "cores": procs, "kind": "port",
            "sample": "%d witnesses of the same workload on %d processes (%.1fs wall); the C oracle "
                      "(oracle/witness_oracle.c, a test-grade restatement; the reference's WASM calculator "
                      "cannot be built or run here)" % (ns, procs, cdt),
            "value_1thread": round(v1, 2), "sample_1thread": "%d witnesses, 1 process (%.1fs)" % (n1, cdt1),
            "host_cpus": nproc, "host_cpus_affinity": affinity,
            # all host cores: one witness per process, no shared state, so the rate scales with
            # processes (16 processes give 14.9-15.2x the 1-thread rate in rounds 1-4); the box allows a one-GPU job
            # 16 busy CPUs, so the nproc-wide figure is the 16-process rate scaled, not a run on every core
            "value_nproc_scaled": round(v * nproc / procs, 2),
            "cores_note": "cores = %d, the host CPU share of a one-GPU job on the GPU box (its OMP_NUM_THREADS); "
                          "value_nproc_scaled = value x %d / %d (the box's nproc), an extrapolation: the pool does "
                          "not allow a one-GPU job to occupy every host core" % (CPU_SHARE, nproc, procs)}
        if args.workload == "poseidon":
            jf = os.path.join(REPO, "profiles", "r5_config1", "poseidon_js.json")
            if os.path.exists(jf):
                js = json.load(open(jf))
                out["cpu_baseline"]["reference_js"] = {
                    k: js.get(k) for k in ("value", "unit", "cores", "sample", "node", "measured_on")}
    return out


def host_delivered(args, inst, sig, n=None):
    """Witnesses delivered into host memory (pzk_witness_stream, include/pzkwit.h): host input rows up, each
    chunk's rows computed, then copied down into pinned host memory while the next chunk computes; the sink
    (this process) checks witness[0] == 1 and the lane status of every row. Reported beside the line, never
    as `value` (which keeps the device-resident definition): it measures the host link, not the kernels."""
    n = n or args.host_sample or max(64, min(4096, int(36e9 // (32 * inst.witness_size))))  # ~36 GB of rows
    rows = make_register_inputs(n, 2 * 10 ** 6, workers=max(1, min(CPU_SHARE, os.cpu_count() or 1)),
                                seed=SIG_SEED[sig], sig=sig)
    seen = {"n": 0, "bad": 0, "one": 0}

    def sink(first, w, st):
        seen["n"] += w.shape[0]
        seen["bad"] += int((st != 0).sum())
        seen["one"] += int((w[:, 0, 0] == 1).sum())

    inst.witness_stream(rows, sink)  # warm: the stream's device slots and pinned host rows are allocated once
    seen.update(n=0, bad=0, one=0)
    t0 = time.perf_counter()
    inst.witness_stream(rows, sink)
    dt = time.perf_counter() - t0
    assert seen["n"] == n, seen
    row_bytes = 32 * inst.witness_size
    link = d2h_link_gbs()
    gbs = n * row_bytes / dt / 1e9
    return {"what": "pzk_witness_stream: inputs from host memory, witnesses into pinned host memory (device->host "
                    "copy of chunk c beside the compute of chunk c + 1), every row handed to a host sink",
            "value": round(n / dt, 2), "unit": "witnesses/s", "witnesses": n, "seconds": round(dt, 3),
            "row_bytes": row_bytes, "layout": "mapped (%s)" % args.sym if args.sym else "O0",
            "gb_per_s": round(gbs, 2),
            "link": {"what": "the host link the rows cross: PCIe 5.0 x16 device->host, 64 GB/s per direction "
                             "theoretical; measured = one 4 GiB device->pinned-host copy on this box",
                     "theoretical_gbs": 64.0, "measured_gbs": link,
                     "frac_of_measured": round(gbs / link, 3) if link else None},
            "sink_checks": {"rows": seen["n"], "status_nonzero": seen["bad"], "witness0_is_one": seen["one"]}}


def d2h_link_gbs(nbytes=4 << 30):
    """Device -> pinned host copy rate of one large buffer (the ceiling host delivery is measured against)."""
    import torch
    try:
        dev = torch.device("cuda", torch.cuda.current_device())
        src = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        dst = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        dst.copy_(src, non_blocking=True)  # warm
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        del src, dst
        return round(nbytes / dt / 1e9, 2)
    except RuntimeError:
        return None


def input_side(sig, distinct=128, n=8192):
    """The input step before the hot path, on the host: EF.SOD files -> this instance's
    input rows with the bulk preprocessor (pzk_passport_inputs) on the host CPU share, rows written into
    resident memory. Reported beside the line; the reference's per-passport processPassport takes ~22 ms
    (Node 12, profiles/r2_passport_preprocessor.json)."""
    from pzkwit import passport as PP, sodgen
    t0 = time.perf_counter()
    key = sodgen.signer_key(sig)
    # SHA-384 signed attributes fit the circuit's one 1024-bit block only without signingTime (sodgen.make_passport)
    uniq = [sodgen.make_passport(sig, key, i, signing_time=sig not in (13, 25)) for i in range(distinct)]
    gen_s = time.perf_counter() - t0
    params = PP.parse(uniq[0])["params"]
    src = PP.sources([uniq[i % distinct] for i in range(n)])
    rows, _ = PP.input_rows(params, uniq[:1])
    rows = np.ones((n,) + rows.shape[1:], dtype=np.uint8)  # resident pages
    t0 = time.perf_counter()
    rows, st = PP.input_rows(params, src, threads=CPU_SHARE, out=rows)
    dt = time.perf_counter() - t0
    return {"what": "EF.SOD + DG1 + DG15 -> input rows (pzk_passport_inputs, include/pzkpassport.h)",
            "passports_per_s": round(n / dt, 1), "threads": CPU_SHARE, "passports": n, "ok": int((st == 0).sum()),
            "row_bytes": int(rows[0].nbytes), "params": params,
            "sample": "%d distinct synthetic SOD passports (pzkwit/sodgen.py, SIGNATURE_TYPE %d; %.1fs to make) repeated"
                      % (distinct, sig, gen_s)}


# ----------------------------------------------------------------------------- config 5
MIX = ((1, 0.4), (2, 0.3), (20, 0.3))  # RSA-2048 / RSA-4096 / ECDSA secp256r1


def _mixed_plan(per_gpu, world):
    """Deterministic config-5 job (every rank derives the same): flow of each of the world x per_gpu
    witnesses (seed 5), the flows' instance parameters, and each rank's cost-balanced contiguous shard."""
    from pzkwit import inputs as I, mixed
    total = per_gpu * world
    rng = np.random.default_rng(5)
    sigs = rng.choice([m[0] for m in MIX], size=total, p=[m[1] for m in MIX])
    flows = {sg: dict(I.CANONICAL, sig=int(sg)) for sg, _ in MIX}
    costs = [mixed.witness_cost(flows[int(sg)]) for sg in sigs]
    shards = [mixed.shard_by_cost(costs, world, r) for r in range(world)]
    return sigs, flows, costs, shards


def _mixed_groups(sigs, lo, hi):
    """A shard's witnesses grouped per flow (MIX order), each group in global order: {sig: [index]}"""
    groups = {}
    for sg, _ in MIX:
        idx = [i for i in range(lo, hi) if int(sigs[i]) == sg]
        if idx:
            groups[sg] = idx
    return groups


def _mixed_host_rows(sigs, lo, hi, n_in_max, workers):
    """Input rows of shard [lo, hi) on the host, grouped per flow (the _mixed_groups order), each row
    zero-padded to n_in_max elements: [hi - lo, n_in_max, 32]"""
    from pzkwit import inputs as I
    n_keys = {1: 64, 2: 8, 20: 64}
    out = np.zeros((hi - lo, n_in_max, 32), dtype=np.uint8)
    pos = 0
    for sg, idx in _mixed_groups(sigs, lo, hi).items():
        where = {gi: pos + k for k, gi in enumerate(idx)}
        n_in = I.PassportGen.shared(5, n_keys[sg], sg).n_inputs
        step = max(1, (len(idx) + workers * 4 - 1) // (workers * 4))
        # a flow's items are not contiguous in the global batch: generate each covering range, keep members
        jobs = [(5, idx[a], idx[min(len(idx), a + step) - 1] + 1, n_keys[sg], sg) for a in range(0, len(idx), step)]
        with I.process_pool(workers) as ex:
            for first, arr in ex.map(_gen_slice, jobs):
                for k in range(len(arr)):
                    gi = first + k
                    if gi in where:
                        out[where[gi], :n_in] = arr[k]
        pos += len(idx)
    return out


class MixedGpuEngine:
    """Config 5's measured path on one rank: one libpzkwit instance per flow, each with its own output slot, so
    the flows' pipelined calls overlap (no synchronisation between instances inside a step)."""

    def __init__(self, flows, groups, dev):
        import torch
        from pzkwit import native
        self.torch, self.dev, self.groups = torch, dev, groups
        self.inst = {sg: native.Instance(native.PZK_CIRCUIT_REGISTER, 0, flows[sg]) for sg in groups}
        self.n_inputs = {sg: i.n_inputs for sg, i in self.inst.items()}
        self.witness_size = {sg: i.witness_size for sg, i in self.inst.items()}

    def setup(self, d_in, first, n_local):
        """d_in: {flow: its compact input rows [n, n_inputs * 32] on the device}; first: {flow: row of its first
        witness in the rank's status vector}."""
        torch = self.torch
        self.d_in, self.first = d_in, first
        # one output slot per flow, sized so the slots and the instances' scratch fit beside each other
        free, _ = torch.cuda.mem_get_info(self.dev)
        scratch = {1: 1 << 20, 2: 2 << 20, 20: 10 << 20}  # per-witness core scratch of one set
        budget = int(free * 0.85) // max(1, len(self.groups))
        self.sub = {sg: max(1, min(len(self.groups[sg]), budget // (32 * self.witness_size[sg] + 3 * scratch[sg])))
                    for sg in self.groups}
        self.d_out = {sg: torch.empty(self.sub[sg] * 32 * self.witness_size[sg], dtype=torch.uint8, device=self.dev)
                      for sg in self.groups}
        self.d_st = torch.zeros(n_local, dtype=torch.int32, device=self.dev)
        torch.cuda.synchronize(self.dev)  # the library's streams do not wait for torch's stream

    def _calls(self):
        """(flow, first row) of every call of a step: flow by flow (PZK_MIX_ORDER=flow) or round robin over the flows
        (default), so each flow's calls are spread over the step instead of one flow's calls all queued first"""
        if os.environ.get("PZK_MIX_ORDER", "rr") == "flow":
            return [(sg, a) for sg, idx in self.groups.items() for a in range(0, len(idx), self.sub[sg])]
        # the flow with the largest witnesses (ECDSA: the longest core chain per call) first in every round
        order = sorted(self.groups, key=lambda sg: -self.witness_size[sg])
        per = {sg: list(range(0, len(self.groups[sg]), self.sub[sg])) for sg in order}
        out, k = [], 0
        while any(k < len(aa) for aa in per.values()):
            out += [(sg, aa[k]) for sg, aa in per.items() if k < len(aa)]
            k += 1
        return out

    def _run(self, st, collect=None):
        for sg, a in self._calls():
            idx = self.groups[sg]
            W, NIN = self.witness_size[sg], self.n_inputs[sg]
            n = min(self.sub[sg], len(idx) - a)
            self.inst[sg].witness_batch_device(self.d_in[sg].data_ptr() + a * NIN * 32, n, self.d_out[sg].data_ptr(),
                                               32 * W, st.data_ptr() + 4 * (self.first[sg] + a))
            if collect:
                self.inst[sg].sync()
                collect(sg, a, n, self.d_out[sg].view(self.sub[sg], W, 32)[:n])

    def step(self):
        self._run(self.d_st)

    def sync(self):
        for i in self.inst.values():
            i.sync()
        self.torch.cuda.synchronize(self.dev)

    def statuses(self):
        return self.d_st

    def public_pass(self, n_pub):
        """Untimed: status + public signals (witness[1 .. n_pub]) of every witness of the shard."""
        torch = self.torch
        st = torch.zeros_like(self.d_st)
        pub = torch.zeros((st.shape[0], n_pub, 32), dtype=torch.uint8, device=self.dev)

        def collect(sg, a, n, rows):
            pub[self.first[sg] + a: self.first[sg] + a + n] = rows[:, 1: 1 + n_pub]
        self._run(st, collect)
        torch.cuda.synchronize(self.dev)
        return st, pub


def run_mixed_rank(args, rank, world, local, dist, engine_cls=MixedGpuEngine, device="cuda", rows_fn=None):
    """One rank of config 5 (also driven by tests/test_host.py over gloo with a stub engine and stub rows).

    Every rank derives the same plan (_mixed_plan: flows, costs, cost-balanced contiguous shards). Rank 0 makes
    every shard's input rows (grouped per flow, zero-padded to the widest flow) and scatters shard r to rank r;
    each rank cuts its flows' compact rows back out, runs W + K steps, and status + public signals are
    all-gathered after the timed region (rank-major; within a rank grouped per flow). Returns the JSON record."""
    import torch
    from pzkwit import native, dist as D
    dev = torch.device(device, local) if device == "cuda" else torch.device(device)
    rows_fn = rows_fn or _mixed_host_rows
    per_gpu = args.batch or 4096
    total = per_gpu * world
    sigs, flows, costs, shards = _mixed_plan(per_gpu, world)
    lo, hi = shards[rank]
    groups = _mixed_groups(sigs, lo, hi)
    engine = engine_cls(flows, groups, dev)
    n_in_max = max(native.layout_inputs(flows[sg]) for sg, _ in MIX)
    row_bytes = n_in_max * 32
    rows_max = max(h - l for l, h in shards)
    t0 = time.time()
    recv = torch.zeros(rows_max * row_bytes, dtype=torch.uint8, device=dev)
    if rank == 0:
        workers = max(1, min(CPU_SHARE * world, os.cpu_count() or 1))
        parts = []
        for r, (a, b) in enumerate(shards):
            h = np.zeros((rows_max, n_in_max, 32), dtype=np.uint8)
            h[: b - a] = rows_fn(sigs, a, b, n_in_max, workers)
            parts.append(torch.from_numpy(h.reshape(-1)))
        log("mixed inputs: %d x %d rows generated on rank 0 in %.1fs" % (world, rows_max, time.time() - t0))
        if dist is None:
            recv.copy_(parts[0])
        else:
            parts = [p.to(dev) for p in parts]
    else:
        parts = None
    if dist is not None:
        dist.scatter(recv, parts, src=0)
    del parts
    view = recv.view(rows_max, row_bytes)
    d_in, first = {}, {}
    pos = 0
    for sg, idx in groups.items():  # per flow: compact rows of its own width
        d_in[sg] = view[pos: pos + len(idx), : 32 * engine.n_inputs[sg]].contiguous()
        first[sg] = pos
        pos += len(idx)
    del recv, view
    engine.setup(d_in, first, hi - lo)
    log("mixed rank %d: flows %s, sub-batches %s" % (rank, {k: len(v) for k, v in groups.items()},
                                                       getattr(engine, "sub", None)))
    for _ in range(args.warmup):
        engine.step()
    engine.sync()
    if dist:
        dist.barrier()
    engine.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        engine.step()
    engine.sync()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    bad = int((engine.statuses() != 0).sum().item())  # lanes failing in the last timed step
    n_pub = 5
    st, pub = engine.public_pass(n_pub)
    my_bytes = sum(costs[lo:hi])
    if dist:
        tt = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        bt = torch.tensor([bad], device=dev, dtype=torch.int64)
        dist.all_reduce(bt)
        bad = int(bt.item())
        st, pub = D.gather_results(dist, st, pub, device=dev)
    import hashlib
    gathered = {"witnesses": int(st.shape[0]), "status_nonzero": int((st != 0).sum().item()),
                "public_sha256": hashlib.sha256(pub.cpu().numpy().tobytes()).hexdigest()[:16],
                "order": "rank-major; within a rank grouped per flow (SIG 1, 2, 20), global order inside a group"}
    value = total * args.steps / dt
    job_gbs = sum(costs) * args.steps / dt / 1e9
    return {
        "metric": "mixed-flow registerIdentityBuilder witnesses/sec (config 5: RSA-2048/RSA-4096/ECDSA-P256)",
        "value": round(value, 2), "unit": "witnesses/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": "mixed flows %s, %d per GPU, cost-sharded" % (dict(MIX), per_gpu),
                   "flows": {str(k): len(v) for k, v in groups.items()}, "rank0_bytes": my_bytes,
                   "sub_batches": {str(k): v for k, v in (getattr(engine, "sub", None) or {}).items()},
                   "invalid_lanes": bad, "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                   "call_order": os.environ.get("PZK_MIX_ORDER", "rr"),
                   "inputs": "rank 0 generates every shard and scatters it (process group)", "gathered": gathered},
        "job_hbm": {"achieved": round(job_gbs, 1), "unit": "GB/s", "frac": round(job_gbs / (HBM_PEAK_GBS * world), 4)},
    }


def bench_mixed(args):
    """Config 5: a mixed-flow batch (40 % RSA-2048, 30 % RSA-4096, 30 % ECDSA secp256r1, seed 5),
    --batch witnesses per GPU on average, sharded across ranks by .wtns bytes (pzkwit.mixed)."""
    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    out = run_mixed_rank(args, rank, world, local, dist)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
