"""ctypes binding of libboojum_mi355x.so (include/boojum_mi355x.h).

This is the product's only route to compute: there is no CPU fallback.  If the
library is missing, importing a compute entry point raises immediately.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libboojum_mi355x.so")

_u64 = ctypes.c_uint64
_u32 = ctypes.c_uint32
_sz = ctypes.c_size_t
_int = ctypes.c_int
_vp = ctypes.c_void_p
_u64p = ctypes.POINTER(ctypes.c_uint64)
# bj_exchange_fn (include/boojum_mi355x.h): int (*)(void* user, int kind, const void* send, void* recv,
# size_t bytes, void* stream)
EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_size_t, ctypes.c_void_p)

# name -> argtypes (restype int unless noted).  Every symbol the header declares.
SIGNATURES = {
    "bj_last_error": ([], ctypes.c_char_p),
    "bj_abi_version": ([], _u32),
    "bj_experiment_knob": ([ctypes.c_char_p, _u64p], _int),
    "bj_release_workspace": ([], _int),
    "bj_release_tables": ([], _int),
    "bj_prepare": ([_u32], _int),
    "bj_precompute_twiddles_d": ([_u32, _int, _vp, _vp], _int),
    "bj_precompute_twiddles_h": ([_u32, _int, _u64p], _int),
    "bj_precompute_twiddles_natural_d": ([_u32, _int, _vp, _vp], _int),
    "bj_bitreverse_enumeration_d": ([_vp, _u32, _sz, _u32, _vp], _int),
    "bj_distribute_powers_d": ([_vp, _u32, _sz, _u32, _u64, _vp], _int),
    "bj_distribute_powers_h": ([_u64p, _sz, _u64], _int),
    "bj_fft_natural_to_bitreversed_d": ([_vp, _u32, _sz, _u32, _u64, _vp, _vp], _int),
    "bj_fft_natural_to_bitreversed_h": ([_u64p, _sz, _u64], _int),
    "bj_ifft_natural_to_natural_d": ([_vp, _u32, _sz, _u32, _u64, _vp, _vp], _int),
    "bj_ifft_natural_to_natural_h": ([_u64p, _sz, _u64], _int),
    "bj_lde_d": ([_vp, _u32, _sz, _u32, _u32, _vp, _vp, _vp], _int),
    "bj_lde_ex_d": ([_vp, _u32, _sz, _u32, _u32, _vp, _vp, _u32, _vp], _int),
    "bj_monomials_to_lde_d": ([_vp, _u32, _sz, _u32, _u32, _vp, _vp], _int),
    "bj_lde_coeffs_d": ([_vp, _u32, _sz, _u32, _vp, _sz, _vp], _int),
    "bj_lde_shard_d": ([_vp, _u32, _sz, _u32, _u32, _u32, _u32, _vp, _vp, _vp], _int),
    "bj_lde_fold_shards_d": ([_vp, _u32, _sz, _u32, _u32, _u32, _vp, _sz, _vp], _int),
    "bj_lde_shard_folded_d": ([_vp, _u32, _sz, _u32, _u32, _u32, _u32, _vp, _vp], _int),
    "bj_poseidon2_permute_d": ([_vp, _sz, _vp], _int),
    "bj_poseidon2_permute_h": ([_u64p], _int),
    "bj_hash_into_leaf_h": ([_u64p, _sz, _u64p], _int),
    "bj_hash_into_node_h": ([_u64p, _u64p, _u64p], _int),
    "bj_merkle_leaves_d": ([_vp, _u32, _sz, _sz, _vp, _vp], _int),
    "bj_merkle_leaves_partial_d": ([_vp, _u32, _sz, _sz, _vp, _vp, _int, _vp], _int),
    "bj_merkle_leaves_chunked_d": ([_vp, _u32, _sz, _sz, _u32, _vp, _vp], _int),
    "bj_merkle_nodes_d": ([_vp, _sz, _u32, _vp, _vp], _int),
    "bj_blake2s_leaves_d": ([_vp, _u32, _sz, _sz, _vp, _vp], _int),
    "bj_blake2s_leaves_chunked_d": ([_vp, _u32, _sz, _sz, _u32, _vp, _vp], _int),
    "bj_blake2s_nodes_d": ([_vp, _sz, _u32, _vp, _vp], _int),
    "bj_blake2s_leaves_partial_d": ([_vp, _u32, _sz, _sz, _u64, _vp, _vp, _int, _vp], _int),
    "bj_blake2s_leaf_h": ([_u64p, _sz, _u64p], _int),
    "bj_keccak256_leaves_d": ([_vp, _u32, _sz, _sz, _vp, _vp], _int),
    "bj_keccak256_leaves_chunked_d": ([_vp, _u32, _sz, _sz, _u32, _vp, _vp], _int),
    "bj_keccak256_nodes_d": ([_vp, _sz, _u32, _vp, _vp], _int),
    "bj_keccak256_leaf_h": ([_u64p, _sz, _u64p], _int),
    "bj_keccak256_node_h": ([_u64p, _u64p, _u64p], _int),
    "bj_blake2s_node_h": ([_u64p, _u64p, _u64p], _int),
    "bj_lde_commit_d": ([_vp, _u32, _sz, _u32, _u32, _u32, _u32, _vp, _vp, _vp, _vp, _u64p, _vp], _int),
    "bj_lde_commit_ex_d": ([_vp, _u32, _sz, _u32, _u32, _u32, _u32, _vp, _vp, _vp, _vp, _u64p, _u32, _vp], _int),
    "bj_lde_commit_h": ([_u64p, _u32, _u32, _u32, _u32, _u32, _u64p, _u64p, _u64p, _u64p], _int),
    "bj_comm_rccl_unique_id": ([_vp], _int),
    "bj_comm_init_rccl": ([_vp, _int, _int, ctypes.POINTER(_vp)], _int),
    "bj_comm_wrap_rccl": ([_vp, _int, _int, ctypes.POINTER(_vp)], _int),
    "bj_comm_local_group_create": ([_int, ctypes.POINTER(_vp)], _int),
    "bj_comm_local_group_destroy": ([_vp], _int),
    "bj_comm_init_local": ([_vp, _int, ctypes.POINTER(_vp)], _int),
    "bj_comm_init_callback": ([_int, _int, EXCHANGE_FN, _vp, _int, ctypes.POINTER(_vp)], _int),
    "bj_comm_destroy": ([_vp], _int),
    "bj_comm_exchange_d": ([_vp, _int, _vp, _vp, _sz, _vp], _int),
    "bj_comm_set_timing": ([_vp, _int], _int),
    "bj_comm_phase_ms": ([_vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(_int)], _int),
    "bj_comm_info": ([_vp, _vp], _int),
    "bj_comm_check_world": ([_vp, _vp, _vp], _int),
    "bj_sharded_columns": ([_u32, _u32, _u32, _int, ctypes.POINTER(_u32)], _int),
    "bj_sharded_commit_d": ([_vp, _vp, _sz, _u32, _u32, _u32, _u32, _u32, _int, _vp, _vp, _vp, _vp, _vp], _int),
    "bj_sharded_query_h": ([_vp, _vp, _vp, _vp, _u32, _u32, _u32, _u32, _u32, _int, _u64, _u64p, _u64p, _u64p,
                            _vp], _int),
    "bj_fri_fold_d": ([_vp, _vp, _sz, _vp, _u64, _u64, _u64, _vp, _vp, _vp], _int),
    "bj_fill_synthetic_d": ([_vp, _u32, _sz, _u32, _u64, _u64, _vp], _int),
    "bj_gl_op_d": ([_int, _vp, _vp, _vp, _sz, _vp], _int),
}



class CommInfo(ctypes.Structure):
    """bj_comm_info_t (include/boojum_mi355x.h), 128 bytes."""
    _fields_ = [("kind", ctypes.c_int32), ("world", ctypes.c_int32), ("rank", ctypes.c_int32),
                ("transport_count", ctypes.c_int32), ("transport_rank", ctypes.c_int32),
                ("device", ctypes.c_int32), ("pci_bus_id", ctypes.c_char * 32), ("host", ctypes.c_char * 64),
                ("reserved", ctypes.c_int32 * 2)]

    KINDS = {0: "rccl", 1: "local", 2: "callback"}

    def as_dict(self):
        return {"kind": self.KINDS.get(self.kind, self.kind), "world": self.world, "rank": self.rank,
                "transport_count": self.transport_count, "transport_rank": self.transport_rank,
                "device": self.device, "pci_bus_id": self.pci_bus_id.decode(errors="replace"),
                "host": self.host.decode(errors="replace")}


assert ctypes.sizeof(CommInfo) == 128

_LIB = None


class BoojumError(RuntimeError):
    pass


def load():
    """Load the HIP library (raises if it is not built: no fallback path exists)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise BoojumError(
                "libboojum_mi355x.so not found at %s -- build it with "
                "`make -C era-boojum_amd` (or __graft_entry__.build())" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _LIB = L
    return _LIB


def check(rc, what=""):
    if rc != 0:
        msg = load().bj_last_error()
        raise BoojumError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))


def call(name, *args):
    check(getattr(load(), name)(*args), name)
