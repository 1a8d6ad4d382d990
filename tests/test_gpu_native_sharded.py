"""GPU parity of the native collective commit (bj_sharded_commit_d).

G ranks run as G threads on one card with the in-process transport (bj_comm_local_*), which
drives exactly the native pipeline (chunked exchange on a second stream, per-chunk LDE and
sponge continuation, subtree, cap gather) with device-to-device copies in place of RCCL.
Every rank's LDE slice, leaves, subtree levels and cap must equal the oracle's single-process
commit, bit for bit.  The RCCL transport itself is exercised at world 1 here (one GPU per rank
is needed beyond that; bench.py --native runs it at N > 1)."""
import threading

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_mod():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    import boojum_amd
    boojum_amd.load()
    return torch


def reference(n_cols, log_n, log_lde, cap, hasher, log_k=None):
    """The oracle's commit: LDE at D (flat (C, n D)), tree over the first k cosets."""
    log_k = log_lde if log_k is None else log_k
    x = O.synthetic_trace(n_cols, log_n)
    nd, nl = 1 << (log_n + log_lde), 1 << (log_n + log_k)
    if hasher == "poseidon2":
        ref = O.lde_commit(x, log_lde, cap, threads=8, log_k=log_k)
    else:
        _, lde = O.lde(x, log_lde, threads=8)
        leaves, nodes, _, cap_ref = O.merkle_construct(np.ascontiguousarray(lde.reshape(n_cols, nd)[:, :nl]), cap,
                                                       threads=8, hasher=hasher)
        ref = {"lde": lde, "leaves": leaves, "nodes": nodes, "cap": cap_ref}
    ref["lde"] = ref["lde"].reshape(n_cols, nd)
    ref["nl"] = nl
    return ref


def check_queries(ref, cap, qs, hasher):
    """OracleQuery::construct results (every rank the same) against the full tree's proofs."""
    nl = ref["nl"]
    levels = (nl.bit_length() - 1) - (cap.bit_length() - 1)
    for idx, (elems, leaf, proof) in zip(query_indices(nl), qs):
        want_leaf, want_path = O.merkle_get_proof(ref["leaves"], ref["nodes"], levels, idx)
        assert np.array_equal(elems, ref["lde"][:, idx]), "query %d elements" % idx
        assert np.array_equal(leaf, want_leaf), "query %d leaf" % idx
        assert np.array_equal(proof, want_path), "query %d path" % idx
        assert O.verify_proof_over_cap(proof, ref["cap"], leaf, idx, hasher=hasher)


def check_rank(ref, P, world, cap, lde, leaves, nodes, cap_got, qs=None, hasher="poseidon2"):
    if qs is not None:
        check_queries(ref, cap, qs, hasher)
    nl, nd = ref["nl"], ref["lde"].shape[1]
    m = nl // world
    # lde (B, C, m): block j is range j G + P of the D-coset domain (cosets [j k, (j+1) k))
    assert lde.shape[0] == nd // nl
    for j in range(nd // nl):
        lo = j * nl + P * m
        assert np.array_equal(lde[j], ref["lde"][:, lo:lo + m]), "rank %d lde block %d" % (P, j)
    assert np.array_equal(leaves, ref["leaves"][P * m:(P + 1) * m]), "rank %d leaves" % P
    assert np.array_equal(cap_got, ref["cap"]), "rank %d cap" % P
    # local subtree level k is the P-th slice of global level k
    glob_off, o, k = [], 0, 1
    while (nl >> k) >= cap:
        glob_off.append(o)
        o += nl >> k
        k += 1
    lo, k = 0, 1
    while (m >> k) >= max(1, cap // world):
        cnt = m >> k
        want = ref["nodes"][glob_off[k - 1] + P * cnt: glob_off[k - 1] + (P + 1) * cnt]
        assert np.array_equal(nodes[lo:lo + cnt], want), "rank %d node level %d" % (P, k)
        lo += cnt
        k += 1
    assert lo == nodes.shape[0]


def query_indices(nl):
    return sorted({0, 1, nl // 2 - 1, nl // 2, nl - 1, (nl * 3) // 7})


def run_local(torch, world, n_cols, log_n, log_lde, cap, hasher, log_k=None):
    from boojum_amd._lib import call
    from boojum_amd.field import stream_of, to_host
    from boojum_amd.sharded import LocalGroup, native_columns, native_sharded_commit, native_sharded_query
    n = 1 << log_n
    trace = torch.empty((n_cols, n), dtype=torch.int64, device="cuda")
    call("bj_fill_synthetic_d", trace.data_ptr(), n_cols, n, log_n, 42, 0, stream_of(trace))
    torch.cuda.synchronize()
    group = LocalGroup(world)
    outs, errors = [None] * world, []

    def rank_main(P):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                cols = torch.tensor(native_columns(n_cols, world, P, hasher), device="cuda")
                shard = trace.index_select(0, cols).contiguous()
                comm = group.comm(P)
                r = native_sharded_commit(comm, shard, n_cols, log_n, log_lde, cap, hasher, log_commit_cosets=log_k)
                s.synchronize()
                lk = log_lde if log_k is None else log_k
                qs = [native_sharded_query(comm, r, n_cols, log_n, log_lde, cap, i, hasher, log_commit_cosets=log_k)
                      for i in query_indices(1 << (log_n + lk))]
                outs[P] = tuple(to_host(t) for t in (r.lde, r.leaves, r.nodes, r.cap)) + (qs,)
                comm.close()
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append((P, repr(e)))

    threads = [threading.Thread(target=rank_main, args=(P,), daemon=True) for P in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in threads), "a rank did not finish"
    group.close()
    assert not errors, errors
    return outs


@pytest.mark.parametrize("world,cfg", [
    (1, (16, 13, 1, 16, "poseidon2")),
    (2, (16, 13, 1, 16, "poseidon2")),   # G == D, pipelined (4, 4 columns per rank)
    (4, (16, 13, 1, 16, "poseidon2")),   # G > D: sender-side fold + all-to-all
    (8, (32, 13, 2, 4, "poseidon2")),    # G > D, cap < G: roots gathered, top levels everywhere
    (2, (32, 13, 2, 16, "poseidon2")),   # G < D: whole cosets
    (8, (24, 12, 2, 16, "poseidon2")),   # 3 columns per rank, chunks 1, 1, 1; DIF-size NTT
    (4, (12, 13, 1, 16, "poseidon2")),   # 3 columns per rank (not a multiple of 2): one chunk
    (8, (256, 13, 2, 16, "poseidon2")),  # C3's column deal at G = 8 (1, 1, 2, 4, 8, 16 per rank)
    (2, (16, 13, 2, 16, "blake2s")),     # chaining value carried across chunks
    (8, (16, 13, 1, 4, "blake2s")),
    (4, (16, 13, 1, 8, "keccak256")),    # no continuation: one chunk
    # LDE at D, tree over the first k < D cosets (prover.rs:313-347, subset_for_degree)
    (1, (16, 13, 3, 32, "poseidon2", 1)),   # proof.json's ratio: D = 8, k = 2, cap 32
    (2, (16, 13, 3, 32, "poseidon2", 1)),   # G = k: whole cosets of every block
    (4, (16, 13, 3, 32, "poseidon2", 1)),   # k < G <= D: sub-cosets folded at the receiver
    (8, (16, 13, 3, 32, "poseidon2", 1)),   # G = D
    (4, (16, 13, 2, 16, "poseidon2", 0)),   # D = 4, k = 1
    (8, (16, 13, 2, 4, "poseidon2", 0)),    # G > D: sender-side fold per block, cap < G
    (8, (16, 13, 2, 16, "blake2s", 0)),
    # world 1 in the three-pass range: the fused LDE straight from the trace (no inverse phase),
    # all blocks of k cosets in one call
    (1, (16, 18, 2, 16, "poseidon2")),
    (1, (16, 18, 3, 32, "poseidon2", 1)),
    (1, (8, 19, 2, 16, "blake2s", 0)),
    # G = 2 D in the three-pass range: half a coset per rank, the sender's fold
    (8, (16, 18, 2, 16, "poseidon2")),
    (8, (8, 19, 2, 4, "blake2s")),
    # the inverse tail folding from registers (ntt_lde3.hip lde3_inv_fold_kernel; G > D only) at
    # F = G / k = 4 and 8, and over B = D / k = 2 blocks of cosets (targets j G + p)
    (8, (16, 18, 1, 16, "poseidon2")),        # D = k = 2: F = 4, B = 1
    (8, (16, 18, 1, 16, "poseidon2", 0)),     # D = 2, k = 1: F = 8, B = 2
    (8, (16, 18, 2, 16, "poseidon2", 1)),     # D = 4, k = 2: F = 4, B = 2
    (8, (16, 18, 3, 32, "poseidon2", 2)),     # G = D = 8, k = 4: the all-gather path (no fold), B = 2
    # G <= D in the three-pass range: the monomials all-gathered, whole cosets per rank
    (2, (16, 18, 2, 16, "poseidon2")),
    (4, (16, 18, 2, 16, "poseidon2")),        # one coset per rank
    (4, (16, 19, 3, 32, "blake2s")),          # two cosets per rank
    (2, (16, 18, 3, 32, "poseidon2", 1)),     # G = k < D, B = 4
    # G <= D, every coset committed: a rank's own columns take the inverse tail fused with its
    # cosets' forward stages (bj::lde_own_shard), the others' columns come from the gathered
    # monomials on both sides of the own run
    (4, (12, 18, 2, 16, "poseidon2")),        # 3 columns per rank: one chunk, own run in the middle
    (8, (16, 18, 3, 32, "poseidon2")),        # G = D = 8: one coset per rank
    (2, (24, 19, 3, 16, "blake2s")),          # four cosets per rank, chaining value across chunks
    (2, (16, 18, 2, 16, "keccak256")),        # no continuation: one chunk, own run then the peer's
])
def test_native_sharded_commit_local_ranks(torch_mod, world, cfg):
    n_cols, log_n, log_lde, cap, hasher = cfg[:5]
    log_k = cfg[5] if len(cfg) > 5 else None
    outs = run_local(torch_mod, world, n_cols, log_n, log_lde, cap, hasher, log_k)
    ref = reference(n_cols, log_n, log_lde, cap, hasher, log_k)
    for P in range(world):
        check_rank(ref, P, world, cap, *outs[P], hasher=hasher)


def test_native_sharded_commit_rccl_world1(torch_mod):
    """The RCCL transport end to end at world 1 (ncclCommInitRank with one rank)."""
    torch = torch_mod
    from boojum_amd._lib import call
    from boojum_amd.field import stream_of, to_host
    from boojum_amd.sharded import NativeComm, native_sharded_commit
    n_cols, log_n, log_lde, cap = 16, 13, 2, 16
    comm = NativeComm.rccl_world1()
    try:
        trace = torch.empty((n_cols, 1 << log_n), dtype=torch.int64, device="cuda")
        call("bj_fill_synthetic_d", trace.data_ptr(), n_cols, 1 << log_n, log_n, 42, 0, stream_of(trace))
        r = native_sharded_commit(comm, trace, n_cols, log_n, log_lde, cap)
        torch.cuda.synchronize()
        ref = reference(n_cols, log_n, log_lde, cap, "poseidon2")
        check_rank(ref, 0, 1, cap, to_host(r.lde), to_host(r.leaves), to_host(r.nodes), to_host(r.cap))
    finally:
        comm.close()


def test_native_sharded_commit_phase_timing(torch_mod):
    """bj_comm_set_timing / bj_comm_phase_ms: the timed calls give positive phase times that
    fit inside the call, the count of calls, a fresh sum after each read, and the same
    commitment as an untimed call."""
    torch = torch_mod
    from boojum_amd._lib import call
    from boojum_amd.field import stream_of, to_host
    from boojum_amd.sharded import NativeComm, native_sharded_commit
    n_cols, log_n, log_lde, cap = 32, 14, 2, 16
    comm = NativeComm.rccl_world1()
    try:
        trace = torch.empty((n_cols, 1 << log_n), dtype=torch.int64, device="cuda")
        call("bj_fill_synthetic_d", trace.data_ptr(), n_cols, 1 << log_n, log_n, 42, 0, stream_of(trace))
        plain = to_host(native_sharded_commit(comm, trace, n_cols, log_n, log_lde, cap).cap)
        assert comm.phase_ms() == ({"inverse": 0.0, "lde": 0.0, "leaves": 0.0, "nodes": 0.0}, 0)
        comm.set_timing(True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(2):
            r = native_sharded_commit(comm, trace, n_cols, log_n, log_lde, cap)
        e1.record()
        torch.cuda.synchronize()
        ms, calls = comm.phase_ms()
        assert calls == 2 and all(v > 0 for v in ms.values())
        assert sum(ms.values()) <= e0.elapsed_time(e1) * 1.05
        assert (to_host(r.cap) == plain).all()
        assert comm.phase_ms()[1] == 0
        comm.set_timing(False)
        native_sharded_commit(comm, trace, n_cols, log_n, log_lde, cap)
        torch.cuda.synchronize()
        assert comm.phase_ms()[1] == 0
    finally:
        comm.close()


def test_native_sharded_commit_rejects_bad_shapes(torch_mod):
    torch = torch_mod
    from boojum_amd._lib import BoojumError
    from boojum_amd.sharded import LocalGroup, NativeShardedResult, native_sharded_commit
    group = LocalGroup(2)
    comm = group.comm(0)
    try:
        out = NativeShardedResult(4, 8, 1, 4, 2)
        with pytest.raises(BoojumError):   # cap_size not a power of two
            native_sharded_commit(comm, torch.zeros((2, 256), dtype=torch.int64, device="cuda"), 4, 8, 1, 3,
                                  out=out)
        with pytest.raises(BoojumError):   # lde degree 1
            native_sharded_commit(comm, torch.zeros((2, 256), dtype=torch.int64, device="cuda"), 4, 8, 0, 4,
                                  out=out)
    finally:
        comm.close()
        group.close()


@pytest.mark.slow
@pytest.mark.parametrize("world", [4, 8])
def test_native_sharded_commit_c3_full_size(torch_mod, world):
    """C3 (2^22 x 256, LDE x4, cap 16) through the native collective at G = 4 (all-gather of
    coefficients) and G = 8 (sender-side fold + all-to-all), ranks as threads on one card: every
    rank's LDE slice, leaves and cap equal the one-GPU commit's (itself bit-exact at C2 and
    property-checked at C3 in test_gpu_fullsize.py), compared on the device."""
    torch = torch_mod
    from boojum_amd import commit
    from boojum_amd.sharded import LocalGroup, native_columns, native_sharded_commit
    n_cols, log_n, log_lde, cap = 256, 22, 2, 16
    nl = 1 << (log_n + log_lde)
    m = nl // world
    torch.cuda.empty_cache()
    trace = commit.synthetic_trace(n_cols, log_n)
    ws = commit.witness_commit(trace, 1 << log_lde, cap)
    torch.cuda.synchronize()
    flat = ws.lde.view(n_cols, nl)
    group = LocalGroup(world)
    results, errors = [None] * world, []

    def rank_main(P):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                cols = torch.tensor(native_columns(n_cols, world, P), device="cuda")
                shard = trace.index_select(0, cols).contiguous()
                comm = group.comm(P)
                r = native_sharded_commit(comm, shard, n_cols, log_n, log_lde, cap)
                s.synchronize()
                del shard
                results[P] = (bool(torch.equal(r.lde[0], flat[:, P * m:(P + 1) * m])),
                              bool(torch.equal(r.leaves, ws.leaves[P * m:(P + 1) * m])),
                              bool(torch.equal(r.cap, ws.cap)))
                del r
                comm.close()
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append((P, repr(e)))

    threads = [threading.Thread(target=rank_main, args=(P,), daemon=True) for P in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in threads), "a rank did not finish"
    group.close()
    assert not errors, errors
    for P, (lde_ok, leaves_ok, cap_ok) in enumerate(results):
        assert lde_ok and leaves_ok and cap_ok, "rank %d of %d: lde %s leaves %s cap %s" % (
            P, world, lde_ok, leaves_ok, cap_ok)
    del ws, flat, trace
    torch.cuda.empty_cache()


def test_native_sharded_commit_peer_failure_aborts_group(torch_mod):
    """A rank that rejects its arguments aborts the in-process group: its peer returns an error
    instead of waiting forever at the first exchange (the group is unusable afterwards)."""
    torch = torch_mod
    from boojum_amd._lib import BoojumError
    from boojum_amd.sharded import LocalGroup, native_sharded_commit
    group = LocalGroup(2)
    res = [None, None]

    def rank_main(P):
        torch.cuda.set_device(0)
        comm = group.comm(P)
        try:
            shard = torch.zeros((8, 1 << 13), dtype=torch.int64, device="cuda")
            native_sharded_commit(comm, shard, 16, 13, 1, 16 if P == 0 else 3)   # rank 1: cap not 2^k
            torch.cuda.synchronize()
            res[P] = "ok"
        except BoojumError as e:
            res[P] = str(e)
        finally:
            comm.close()

    threads = [threading.Thread(target=rank_main, args=(P,), daemon=True) for P in range(2)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=60)
    assert not any(t.is_alive() for t in threads), "a rank is still blocked"
    group.close()
    assert "power-of-two" in res[1], res
    assert "peer rank" in res[0], res


@pytest.mark.slow
def test_native_sharded_commit_c4_one_coset_per_rank(torch_mod):
    """C4's intended split (BASELINE configs[3]): 2^23 x 256 at LDE x8 over G = D = 8 ranks, one
    coset per rank, coefficients all-gathered.  Eight ranks do not fit one card at once (16 GiB
    of gathered coefficients + 16 GiB of LDE each), so each rank runs alone through the native
    call with a replay transport: its chunk all-gathers deliver the coefficient columns the
    other ranks would have sent (bj_lde_coeffs_d format, taken from the one-GPU commit's
    monomials), everything else -- its own iNTTs, its coset's LDE, the chained sponge, its
    subtree -- is the product path.  Every rank's LDE, leaves and subtree root pair must equal
    the one-GPU commit's slice, compared on the device; that commit's cap equals the oracle's."""
    import ctypes
    torch = torch_mod
    from boojum_amd import commit
    from boojum_amd._lib import EXCHANGE_FN
    from boojum_amd.sharded import NativeComm, NativeShardedResult, native_columns, native_sharded_commit
    n_cols, log_n, log_lde, cap = 256, 23, 3, 16
    world, n = 8, 1 << 23
    torch.cuda.empty_cache()
    trace = commit.synthetic_trace(n_cols, log_n)
    ws = commit.witness_commit(trace, 1 << log_lde, cap)
    torch.cuda.synchronize()
    # the one-GPU commit itself is pinned to the oracle's C4 cap (tools/make_bench_golden.py
    # --chunk-cols 8), so every rank below is compared with oracle-checked slices
    import json
    import os
    golden = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "bench_caps.json")))["caps"]
    want = [[int(x, 16) for x in row] for row in golden["C4/poseidon2"]["cap"]]
    from boojum_amd.field import to_host
    got = [[int(x) % ((1 << 64) - (1 << 32) + 1) for x in row] for row in to_host(ws.cap)]
    assert got == want, "one-GPU C4 cap differs from the oracle's"
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    mono = ws.scratch  # (C, n): the monomials in bj_lde_coeffs_d's bit-reversed format
    cap_local = cap // world
    for P in range(world):
        state = {"base": None}

        def replay(user, kind, send, recv, nbytes, stream, P=P, state=state):
            assert kind == 0, "G = D exchanges by all-gather"
            if nbytes < 8 * n:   # the cap gather: every rank's cap slice
                src = ws.cap.data_ptr()
                return hip.hipMemcpyAsync(recv, src, world * nbytes, 3, stream)
            if state["base"] is None:
                state["base"] = recv   # chunk 0 starts at column 0
            c0 = (recv - state["base"]) // (8 * n)
            return hip.hipMemcpyAsync(recv, mono[c0].data_ptr(), world * nbytes, 3, stream)

        fn = EXCHANGE_FN(replay)
        comm = NativeComm._make("bj_comm_init_callback", world, P, fn, None, 0, world=world, rank=P, keep=fn)
        try:
            cols = torch.tensor(native_columns(n_cols, world, P), device="cuda")
            shard = trace.index_select(0, cols).contiguous()
            res = NativeShardedResult(n_cols, log_n, log_lde, cap, world)
            native_sharded_commit(comm, shard, n_cols, log_n, log_lde, cap, out=res)
            torch.cuda.synchronize()
            assert torch.equal(res.lde[0], ws.lde[:, P, :]), "rank %d lde (coset %d)" % (P, P)
            assert torch.equal(res.leaves, ws.leaves[P * n:(P + 1) * n]), "rank %d leaves" % P
            assert torch.equal(res.nodes[-cap_local:], ws.cap[P * cap_local:(P + 1) * cap_local]), \
                "rank %d subtree roots" % P
            del shard, res
        finally:
            comm.close()
        torch.cuda.empty_cache()
    del ws, trace, mono
    torch.cuda.empty_cache()


def test_local_exchange_layouts():
    """bj_comm_exchange_d's two layouts over the in-process group at G = 4 (the same calls the
    commit issues per chunk): all-gather recv block p = rank p's send; all-to-all recv block p =
    block `rank` of rank p's send."""
    import torch
    from boojum_amd._lib import call
    from boojum_amd.field import stream_of
    from boojum_amd.sharded import XCHG_ALL_GATHER, XCHG_ALL_TO_ALL, LocalGroup
    world, m = 4, 1000
    group = LocalGroup(world)
    got, errors = [None] * world, []

    def rank_main(P):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                comm = group.comm(P)
                ag_send = torch.arange(m, dtype=torch.int64, device="cuda") + 10**6 * P
                ag_recv = torch.empty(world * m, dtype=torch.int64, device="cuda")
                # all-to-all send block q (destined to rank q) = 10^6 P + 10^3 q + i
                a2a_send = (torch.arange(world * m, dtype=torch.int64, device="cuda") % m
                            + 10**6 * P + 10**3 * (torch.arange(world * m, device="cuda") // m))
                a2a_recv = torch.empty(world * m, dtype=torch.int64, device="cuda")
                for kind, snd, rcv in ((XCHG_ALL_GATHER, ag_send, ag_recv), (XCHG_ALL_TO_ALL, a2a_send, a2a_recv)):
                    call("bj_comm_exchange_d", comm.handle, kind, snd.data_ptr(), rcv.data_ptr(), 8 * m, stream_of(rcv))
                s.synchronize()
                got[P] = (ag_recv.cpu(), a2a_recv.cpu())
                comm.close()
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append((P, repr(e)))

    threads = [threading.Thread(target=rank_main, args=(P,), daemon=True) for P in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=60)
    assert not any(t.is_alive() for t in threads), "a rank did not finish"
    group.close()
    assert not errors, errors
    i = torch.arange(m, dtype=torch.int64)
    for P in range(world):
        ag, a2a = got[P]
        for p in range(world):
            assert torch.equal(ag[p * m:(p + 1) * m], i + 10**6 * p)
            assert torch.equal(a2a[p * m:(p + 1) * m], i + 10**6 * p + 10**3 * P)


@pytest.mark.parametrize("var,value", [("BJ_LEAVES_DEFER", "1"), ("BJ_LEAVES_DEFER", "99"),
                                       ("BJ_INV_FOLD_UNPAIRED", "1"), ("BJ_LEAVES_GROUP", "1"),
                                       ("BJ_LEAVES_GROUP", "3"), ("BJ_LDE_OWN_FUSED", "0")])
def test_native_sharded_commit_env_knobs(torch_mod, var, value):
    """The pipeline's experiment knobs must give the same commitment: BJ_LEAVES_DEFER
    (collective.hip leaves_defer(), read once per process: chunk k's leaves after chunk k + d's
    LDE, or after every LDE), BJ_LEAVES_GROUP (chunks per leaf grid: 1, or 3 instead of the
    default 1), BJ_LDE_OWN_FUSED=0 (G <= D: every column's forward from the gathered monomials
    instead of the own columns' inverse tail fused with their forward) and BJ_INV_FOLD_UNPAIRED (ntt_lde3.hip: the sender fold's
    per-target loop instead of the paired even/odd form, F = 2, 4, 8).  Run in a child process."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = "\n".join([
        # conftest.py's path order: oracle/ (oracle.py), the package, the repo root, then tests/
        "import sys; sys.path[:0] = [%r, %r, %r, %r]" % (os.path.join(os.path.dirname(here), "oracle"),
                                                        os.path.join(os.path.dirname(here), "era-boojum_amd"),
                                                        os.path.dirname(here), here),
        "import torch, boojum_amd; boojum_amd.load()",
        "import test_gpu_native_sharded as T, ctypes",
        "v = ctypes.c_uint64(0); assert boojum_amd._lib.load().bj_experiment_knob(%r, ctypes.byref(v)) == 0" % var.encode(),
        "assert v.value == int(%r), v.value" % value,
        "for world, cfg in [(8, (256, 13, 2, 16, 'poseidon2')), (2, (16, 18, 2, 16, 'poseidon2')),",
        "                   (4, (16, 13, 1, 16, 'poseidon2')), (2, (16, 13, 2, 16, 'blake2s')),",
        "                   (8, (16, 18, 2, 16, 'poseidon2')), (8, (16, 18, 1, 16, 'poseidon2')),",
        "                   (8, (16, 18, 1, 16, 'poseidon2', 0)), (8, (16, 18, 2, 16, 'poseidon2', 1))]:",
        "    outs = T.run_local(torch, world, *cfg)",
        "    ref = T.reference(*cfg)",
        "    for P in range(world):",
        "        T.check_rank(ref, P, world, cfg[3], *outs[P], hasher=cfg[4])",
        "print('knob ok')",
    ])
    env = dict(os.environ, BJ_EXPERIMENTS="1", **{var: value})
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0 and "knob ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
