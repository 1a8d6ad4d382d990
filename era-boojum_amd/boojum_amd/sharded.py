"""Coset-sharded witness commitment across G GPUs (one process per GPU, RCCL over xGMI).

The reference runs the whole commitment on one host (prover.rs:313-353 with the Worker
pool). Its multi-GPU split (BASELINE north_star) is one native collective call
per rank, `bj_sharded_commit_d` (csrc/collective.hip):

  * the trace is column-sharded: every rank holds C/G of the columns, dealt chunk by chunk
    (`native_columns`, bj_sharded_columns) so the exchange of chunk k overlaps the work on the
    chunks before it;
  * each rank inverse-transforms its own columns; G <= D: the coefficients are all-gathered;
    G > D: the sender folds its columns for every rank and all-to-alls deliver them;
  * the tree covers the first k = fri_lde_factor cosets of the D-coset LDE (subset_for_degree,
    prover.rs:325-347); rank P owns leaf range [P m, (P+1) m), m = k n / G, and the same range
    of every other block of k cosets (LDE only), so the LDE work stays balanced;
  * leaves and the subtree over them are hashed locally (contiguous aligned leaf ranges are
    subtrees of the reference's tree); the cap is all-gathered (cap < G: the G subtree roots
    are gathered and the top levels hashed on every rank).

This module is the host side of that call: communicators (`NativeComm`: RCCL, an in-process
group of ranks on one device, or a torch.distributed group through the callback transport),
the output buffers, and the query.  There is one pipeline: the bench, the tests and the
multi-GPU runs all go through `bj_sharded_commit_d`.
"""
import ctypes

import torch

from ._lib import EXCHANGE_FN as _EXCHANGE_FN, call, check, load
from .field import stream_of

HASHER_IDS = {"poseidon2": 0, "blake2s": 1, "keccak256": 2}
XCHG_ALL_GATHER, XCHG_ALL_TO_ALL = 0, 1   # bj_exchange_fn kinds (include/boojum_mi355x.h)


def _log2(n):
    if n <= 0 or n & (n - 1):
        raise ValueError("size must be a power of two, got %d" % n)
    return n.bit_length() - 1


def native_columns(n_cols, world, rank, hasher="poseidon2"):
    """bj_sharded_columns: the global trace columns rank `rank` of `world` holds, in the order of
    its trace-shard rows.  Host logic only (no device call)."""
    log_g = _log2(world)
    out = (ctypes.c_uint32 * (n_cols // world if n_cols % world == 0 and n_cols else 1))()
    check(load().bj_sharded_columns(n_cols, log_g, rank, HASHER_IDS[hasher], out), "bj_sharded_columns")
    return list(out)


class LocalGroup:
    """bj_comm_local_group_*: in-process ranks (threads) sharing one device.  A rehearsal
    transport that runs the native pipeline multi-rank on one GPU; not for performance."""

    def __init__(self, world):
        h = ctypes.c_void_p()
        check(load().bj_comm_local_group_create(world, ctypes.byref(h)), "bj_comm_local_group_create")
        self.handle, self.world = h, world

    def comm(self, rank):
        return NativeComm._make("bj_comm_init_local", self.handle, rank, world=self.world, rank=rank, keep=self)

    def close(self):
        if self.handle:
            load().bj_comm_local_group_destroy(self.handle)
            self.handle = None


def _host_view(addr, nbytes):
    """int64 CPU tensor over host memory the library handed to a callback (no copy)."""
    n = nbytes // 8
    if n == 0:
        return torch.empty((0,), dtype=torch.int64)
    return torch.frombuffer((ctypes.c_int64 * n).from_address(addr), dtype=torch.int64)


class NativeComm:
    """An opaque bj_comm (include/boojum_mi355x.h): the communicator of bj_sharded_commit_d."""

    def __init__(self, handle, world, rank, keep=None):
        self.handle, self.world, self.rank, self._keep = handle, world, rank, keep

    def info(self):
        """bj_comm_info: what the transport reports for this rank (RCCL: ncclCommCount,
        ncclCommUserRank, ncclCommCuDevice), with the device's PCI bus id and the host name."""
        from ._lib import CommInfo
        out = CommInfo()
        check(load().bj_comm_info(self.handle, ctypes.byref(out)), "bj_comm_info")
        return out.as_dict()

    def check_world(self, stream=None):
        """bj_comm_check_world (collective): every rank's info, gathered.  Returns (ok, [info per
        rank], message): ok is False, with the library's message, when the transport's world is not
        this communicator's (count, rank order), when two RCCL ranks drive one device, or when a
        rank could not read its own record (BJ_EINVAL on every rank).  Only a transport or HIP
        error raises BoojumError."""
        from ._lib import BoojumError, CommInfo
        out = (CommInfo * self.world)()
        rc = load().bj_comm_check_world(self.handle, out, stream)
        infos = [r.as_dict() for r in out]
        if rc == 0:
            return True, infos, ""
        msg = load().bj_last_error().decode(errors="replace")
        if rc != -22:
            raise BoojumError("bj_comm_check_world: rc %d: %s" % (rc, msg))
        return False, infos, msg

    @classmethod
    def _make(cls, fn, *args, world, rank, keep=None):
        h = ctypes.c_void_p()
        check(getattr(load(), fn)(*args, ctypes.byref(h)), fn)
        return cls(h, world, rank, keep)

    @classmethod
    def rccl(cls, group=None):
        """A fresh RCCL communicator over the ranks of the torch.distributed group (one process
        per GPU, current device): rank 0 makes the unique id, the group broadcasts it, every rank
        joins (ncclCommInitRank).  Collective."""
        import torch.distributed as dist
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        uid = (ctypes.c_uint8 * 128)()
        if rank == 0:
            check(load().bj_comm_rccl_unique_id(uid), "bj_comm_rccl_unique_id")
        box = [bytes(uid)]
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        uid = (ctypes.c_uint8 * 128).from_buffer_copy(box[0])
        return cls._make("bj_comm_init_rccl", uid, world, rank, world=world, rank=rank)

    @classmethod
    def rccl_world1(cls):
        """A one-rank RCCL communicator (no process group needed)."""
        uid = (ctypes.c_uint8 * 128)()
        check(load().bj_comm_rccl_unique_id(uid), "bj_comm_rccl_unique_id")
        return cls._make("bj_comm_init_rccl", uid, 1, 0, world=1, rank=0)

    @classmethod
    def torch_dist(cls, group=None):
        """The callback transport over a torch.distributed group of any backend (gloo for ranks
        that share a GPU): the library stages each exchange through host memory and this callback
        runs it as a torch collective on CPU tensors.  Every exchange synchronises, so this is a
        rehearsal transport (correctness of the N > 1 pipeline on one card), not a benchmark.  A
        failing exchange aborts the group, so the peers' calls fail promptly too."""
        import torch.distributed as dist
        world, rank = dist.get_world_size(group), dist.get_rank(group)

        def exchange(user, kind, send, recv, nbytes, stream):
            try:
                out = _host_view(recv, world * nbytes)
                if kind == XCHG_ALL_GATHER:
                    src = _host_view(send, nbytes).clone()
                    dist.all_gather(list(out.view(world, -1).unbind(0)), src, group=group)
                else:
                    src = _host_view(send, world * nbytes).clone()
                    dist.all_to_all_single(out, src, group=group)
                return 0
            except Exception:  # noqa: BLE001 - reported through the C return code
                import traceback
                traceback.print_exc()
                # the peers are blocked in the same collective: abort the group so they fail
                # now (gloo: "connection closed by peer") instead of at the group's timeout
                try:
                    (group if group is not None else dist.group.WORLD).abort()
                except Exception:  # noqa: BLE001 - best effort; the error is returned either way
                    pass
                return 1

        fn = _EXCHANGE_FN(exchange)
        return cls._make("bj_comm_init_callback", world, rank, fn, None, 1, world=world, rank=rank, keep=fn)

    @classmethod
    def null(cls, world, rank):
        """A transport whose exchanges move nothing (device-mode callback returning at once): rank
        `rank`'s compute of a G-way commit alone, for timing probes.  Its outputs are not a
        commitment (the received buffers are never filled)."""
        fn = _EXCHANGE_FN(lambda *a: 0)
        return cls._make("bj_comm_init_callback", world, rank, fn, None, 0, world=world, rank=rank, keep=fn)

    def link_probe(self, kind, bytes_per_rank, stream=None, agree=None):
        """Time one bj_comm_exchange_d of `kind` (XCHG_ALL_GATHER / XCHG_ALL_TO_ALL) with
        `bytes_per_rank` bytes per rank block, as bj_sharded_commit_d's exchanges move them
        (collective; every rank calls it).  A small exchange of the same kind first sets up the
        transport's connections; the caller should hold the ranks at a barrier just before.
        `agree(ok) -> bool`, when given, is a host-side collective over the ranks (every rank's
        buffers allocated?): the exchange runs only when every rank could allocate, so one rank's
        allocation failure cannot leave its peers waiting in the transport.  Returns the
        milliseconds between HIP events on `stream` around the exchange -- the transport's time
        plus any wait for peers that reached it later, so the minimum over ranks is the closest to
        the link's own time -- or None when a rank could not allocate."""
        dev = torch.device("cuda", torch.cuda.current_device())
        st = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        world = self.world
        words = max(1, bytes_per_rank // 8)
        nsend = words * (world if kind == XCHG_ALL_TO_ALL else 1)
        try:
            send = torch.zeros(nsend, dtype=torch.int64, device=dev)
            recv = torch.empty(words * world, dtype=torch.int64, device=dev)
            ok = True
        except RuntimeError:  # allocation failure: reported through agree(), never raised alone
            send = recv = None
            ok = False
        if agree is not None:
            ok = agree(ok)
        if not ok:
            return None
        check(load().bj_comm_exchange_d(self.handle, kind, send.data_ptr(), recv.data_ptr(), 8, st),
              "bj_comm_exchange_d")
        torch.cuda.synchronize()
        s_ = torch.cuda.ExternalStream(st) if stream is not None else torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s_)
        check(load().bj_comm_exchange_d(self.handle, kind, send.data_ptr(), recv.data_ptr(), words * 8, st),
              "bj_comm_exchange_d")
        e1.record(s_)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        del send, recv
        return ms

    def set_timing(self, on=True):
        """Record phase events in every later bj_sharded_commit_d call (bj_comm_set_timing)."""
        check(load().bj_comm_set_timing(self.handle, 1 if on else 0), "bj_comm_set_timing")

    def phase_ms(self):
        """Summed ms of the timed calls since the last read: ({inverse, lde, leaves, nodes}, calls)."""
        ms = (ctypes.c_float * 4)()
        calls = ctypes.c_int()
        check(load().bj_comm_phase_ms(self.handle, ms, ctypes.byref(calls)), "bj_comm_phase_ms")
        return dict(zip(("inverse", "lde", "leaves", "nodes"), list(ms))), calls.value

    def close(self):
        if self.handle:
            load().bj_comm_destroy(self.handle)
            self.handle = None


class NativeShardedResult:
    """Rank P's outputs of bj_sharded_commit_d for an LDE at D = 2^log_lde committed over its
    first k = 2^log_commit_cosets cosets (k = D by default): lde (B, C, m) with B = D / k blocks
    (block 0 the committed one, this rank's leaf range), leaves (m, 4), nodes (m - cap_local, 4),
    cap (cap, 4), all int64 on the device; m = k n / G."""

    def __init__(self, n_cols, log_n, log_lde, cap_size, world, device="cuda", log_commit_cosets=None):
        log_k = log_lde if log_commit_cosets is None else log_commit_cosets
        m = ((1 << log_n) << log_k) // world
        cap_local = max(1, cap_size // world)
        kw = dict(dtype=torch.int64, device=device)
        self.m, self.cap_local, self.log_k = m, cap_local, log_k
        self.lde = torch.empty((1 << (log_lde - log_k), n_cols, m), **kw)
        self.leaves = torch.empty((m, 4), **kw)
        self.nodes = torch.empty((m - cap_local, 4), **kw)
        self.cap = torch.empty((cap_size, 4), **kw)


def native_sharded_commit(comm, trace_shard, n_cols, log_n, log_lde, cap_size, hasher="poseidon2", out=None,
                          log_commit_cosets=None):
    """bj_sharded_commit_d on the current stream: this rank's part of the G-way witness commit,
    trace_shard (C/G, n) in native_columns order.  Collective over `comm`."""
    if tuple(trace_shard.shape) != (n_cols // comm.world, 1 << log_n) or trace_shard.stride(1) != 1:
        raise ValueError("trace shard must be (%d, %d) with unit-stride rows" % (n_cols // comm.world, 1 << log_n))
    log_k = log_lde if log_commit_cosets is None else log_commit_cosets
    out = out or NativeShardedResult(n_cols, log_n, log_lde, cap_size, comm.world, trace_shard.device, log_k)
    call("bj_sharded_commit_d", comm.handle, trace_shard.data_ptr(), trace_shard.stride(0), n_cols, log_n, log_lde,
         log_k, cap_size, HASHER_IDS[hasher], out.lde.data_ptr(), out.leaves.data_ptr(), out.nodes.data_ptr(),
         out.cap.data_ptr(), stream_of(out.lde))
    return out


def native_sharded_query(comm, res, n_cols, log_n, log_lde, cap_size, tree_idx, hasher="poseidon2",
                         log_commit_cosets=None):
    """bj_sharded_query_h: OracleQuery::construct on a native sharded commit (res is this rank's
    NativeShardedResult).  Collective over `comm`; every rank returns the same
    (leaf_elements (C,), leaf_hash (4,), proof (depth, 4)) as numpy uint64."""
    import numpy as np
    log_k = log_lde if log_commit_cosets is None else log_commit_cosets
    depth = (log_n + log_k) - _log2(cap_size)
    elems = np.zeros(n_cols, dtype=np.uint64)
    leaf = np.zeros(4, dtype=np.uint64)
    proof = np.zeros((max(depth, 1), 4), dtype=np.uint64)
    p = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))  # noqa: E731
    call("bj_sharded_query_h", comm.handle, res.lde.data_ptr(), res.leaves.data_ptr(), res.nodes.data_ptr(), n_cols,
         log_n, log_lde, log_k, cap_size, HASHER_IDS[hasher], tree_idx, p(elems), p(leaf), p(proof),
         stream_of(res.lde))
    return elems, leaf, proof[:depth]
