"""QueryIdentity(80) on the CPU: the oracle restatement (oracle/query.inc.c) against
independent math on generated queries, its check sites, and the host layout (builder_query.cpp) against the
oracle's sizes. No device is needed."""
import numpy as np
import pytest

from pzkwit import native, query as Q
from pzkwit.field import P, SplitMix64, poseidon


def test_layout_matches_oracle_sizes(oracle):
    nin, nw = oracle.query_sizes()
    assert nin == Q.N_INPUTS == native.layout_inputs({}, circuit=native.PZK_CIRCUIT_QUERY)
    assert nw == native.layout_witness_size({}, circuit=native.PZK_CIRCUIT_QUERY) == 141169
    nin, nw = oracle.query_sizes(td1=True)  # QueryIdentityTD1 (document_type 1)
    assert nin == Q.N_INPUTS_TD1 == native.layout_inputs({"doc": 1}, circuit=native.PZK_CIRCUIT_QUERY)
    assert nw == native.layout_witness_size({"doc": 1}, circuit=native.PZK_CIRCUIT_QUERY) == 143028
    with pytest.raises(native.PzkError):
        native.layout_info({"size_arg": 40}, circuit=native.PZK_CIRCUIT_QUERY)


def test_country_table_is_the_packed_alpha3_codes():
    C = Q.countries()
    assert len(set(C)) == 240 and C[0] == int.from_bytes(b"ABW", "big") and C[-1] == int.from_bytes(b"ZWE", "big")
    assert C == sorted(C)


@pytest.mark.parametrize("seed,td1", [(1, False), (2, False), (3, False), (4, True), (5, True)])
def test_valid_queries_pass_and_outputs_match_math(oracle, seed, td1):
    rng = SplitMix64(0x51 + seed)
    nout, nin = (10, 858) if td1 else (9, 842)
    for k in range(4):
        sel = [0, (1 << 18) - 1, None, 1 | (1 << 5)][k]
        inp, info = Q.make_query(rng, selector=sel, depth=[0, 1, 79, None][k], td1=td1)
        rc, w = oracle.query_witness(Q.pack(inp), td1=td1)
        assert rc == 0
        got = [oracle.from_elem(w[1 + i]) for i in range(nout)]
        assert got == Q.public_outputs(inp, info)
        # independent recomputations: BabyJubJub key, nullifier, the identity-state SMT root
        ax, ay = info["pk_identity"]
        assert (ax * ax * Q.A_BJJ + ay * ay - 1 - Q.D_BJJ * ax * ax * ay * ay) % P == 0
        assert info["nullifier"] == poseidon([inp["skIdentity"], poseidon([inp["skIdentity"]]), inp["eventID"]])
        assert w[0, 0] == 1 and (w[0, 1:] == 0).all()
        # main inputs are copied after the outputs, eventDataSquare after them
        assert (w[1 + nout:1 + nout + nin] == Q.pack(inp)).all()
        assert oracle.from_elem(w[1 + nout + nin]) == inp["eventData"] ** 2 % P


def _fail_case(kind, rng, td1=False):
    if kind == "bound":        # selected timestamp lower bound above the timestamp
        inp, _ = Q.make_query(rng, selector=1 << 8, td1=td1)
        inp["timestampLowerbound"] = inp["timestamp"] + 5
        return inp, 19
    if kind == "date":         # expirationDateLowerbound not a digit string ("24A101"), its check not selected
        inp, _ = Q.make_query(rng, selector=0, td1=td1)
        inp["expirationDateLowerbound"] = int.from_bytes(b"24A101", "big")
        return inp, 20
    if kind == "blacklist":
        inp, info = Q.make_query(rng, selector=0, td1=td1)
        inp["citizenshipMask"] |= 1 << (239 - info["citizenship_index"])
        return inp, 21
    if kind == "unlisted":
        inp, _ = Q.make_query(rng, selector=0, cit_code=b"XXX", td1=td1)
        return inp, 22
    if kind == "root":
        inp, _ = Q.make_query(rng, selector=0, td1=td1)
        inp["idStateRoot"] = (inp["idStateRoot"] + 1) % P
        return inp, 23
    if kind == "smt_last":     # a non-zero last sibling (SMTVerifier.circom:54) before the root check
        inp, _ = Q.make_query(rng, selector=0, depth=3, td1=td1)
        inp["idStateSiblings"][79] = 7
        return inp, 13
    if kind == "selector":     # selector >= 2^18: Num2Bits(18)
        inp, _ = Q.make_query(rng, selector=0, td1=td1)
        inp["selector"] = 1 << 20
        return inp, 1
    raise ValueError(kind)


FAIL_KINDS = ["bound", "date", "blacklist", "unlisted", "root", "smt_last", "selector"]


@pytest.mark.parametrize("td1", [False, True])
@pytest.mark.parametrize("kind", FAIL_KINDS)
def test_check_sites(oracle, kind, td1):
    inp, code = _fail_case(kind, SplitMix64(0x77 + FAIL_KINDS.index(kind)), td1)
    rc, _ = oracle.query_witness(Q.pack(inp), td1=td1)
    assert rc == code


def test_unselected_bounds_do_not_fail(oracle):
    rng = SplitMix64(0x99)
    inp, _ = Q.make_query(rng, selector=(1 << 18) - 1 - (1 << 8))
    inp["timestampLowerbound"] = inp["timestamp"] + 5
    rc, w = oracle.query_witness(Q.pack(inp))
    assert rc == 0


# the constraint that each check site violates (template, reference line), as the checker names it
FAIL_CONSTRAINT = {"bound": ("ForceEqualIfEnabled", 42), "date": ("DateDecoder", 22),
                   "blacklist": ("CitizenshipCheck", 271), "unlisted": ("CitizenshipCheck", 274),
                   "root": ("IdentityStateVerifier", 46), "smt_last": ("SMTLevIns", None), "selector": ("Num2Bits", 26)}


@pytest.mark.parametrize("td1", [False, True])
def test_constraints_hold_on_oracle_witnesses(oracle, td1):
    """The independent constraint checker (oracle/r1cs_query.inc.c, restated from the .circom constraints, never
    computing a witness) accepts oracle witnesses: every constraint holds and every signal is read by one."""
    import pyr1cs
    rng = SplitMix64(0xC0)
    for sel, depth in ((0, 0), ((1 << 18) - 1, 79), (None, None)):
        inp, _ = Q.make_query(rng, selector=sel, depth=depth, td1=td1)
        rc, w = oracle.query_witness(Q.pack(inp), td1=td1)
        assert rc == 0
        crc, rep = pyr1cs.check_query(w, td1=td1)
        assert crc == 0 and rep["n_failed"] == 0 and rep["n_uncovered"] == 0, rep
        assert rep["size_walked"] == w.shape[0]
        if not td1:
            assert rep["n_constraints"] == 140542


@pytest.mark.parametrize("kind", FAIL_KINDS)
def test_checker_names_the_failing_constraint(oracle, kind):
    import pyr1cs
    inp, code = _fail_case(kind, SplitMix64(0x77 + FAIL_KINDS.index(kind)))
    rc, w = oracle.query_witness(Q.pack(inp))
    assert rc == code
    crc, rep = pyr1cs.check_query(w)
    assert crc == 1 and rep["n_failed"] >= 1
    tmpl, line = FAIL_CONSTRAINT[kind]
    assert rep["first_template"].startswith(tmpl), rep
    if line is not None:
        assert rep["first_line"] == line, rep
