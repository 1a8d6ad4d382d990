"""CPU steps of the sharded-commit model (tests/sharded_model.py), built on the oracle -- TEST ONLY.

Lets the multi-process (gloo) tests exercise the schedule of the native collective commit
(column shards, exchange order, leaf-range ownership, cap assembly incl. cap < G) on CPU
tensors.  Each step restates the contract of the C-ABI entry point the native call uses
(include/boojum_mi355x.h: bj_lde_coeffs_d, bj_lde_shard_d, bj_lde_fold_shards_d,
bj_lde_shard_folded_d, bj_merkle_*_d)."""
import numpy as np

import oracle as O


def _np(t):
    return t.numpy().view(np.uint64)


class CpuShardOps:
    def __init__(self, hasher="poseidon2"):
        self.hasher = hasher

    def prepare(self, log_n):
        pass

    def synthetic(self, out, log_n, first_col):
        _np(out)[:] = O.synthetic_trace(out.shape[0], log_n, col_offset=first_col)

    def coeffs(self, trace, out, log_n):
        # monomials in bit-reversed order
        for c in range(trace.shape[0]):
            _np(out)[c] = O.bitreverse(O.ifft_natural_to_natural(_np(trace)[c]))

    @staticmethod
    def _shard_shift(log_n, log_lde, log_shards, shard):
        # s' = 7 * w_{nD}^{bitrev_{log G}(P)}
        br = int(O.bitreverse(np.arange(1 << log_shards, dtype=np.uint64))[shard])
        return O.gl_mul(O.gl_pow(O.domain_generator(log_n + log_lde), br), 7)

    def fold_shards(self, coeffs, log_n, log_lde, log_shards, out, shards=None):
        # h_t = sum_a c_{t+am} (s_P^m)^a for every listed shard P (default all), out[i] for
        # shards[i]; stored bit-reversed like the input
        n = 1 << log_n
        m = (n << log_lde) >> log_shards
        f = n // m
        shards = list(range(1 << log_shards)) if shards is None else list(shards)
        for i, P in enumerate(shards):
            z = O.gl_pow(self._shard_shift(log_n, log_lde, log_shards, P), m)
            for c in range(coeffs.shape[0]):
                mono = [int(x) for x in O.bitreverse(_np(coeffs)[c])]
                h = []
                for t in range(m):
                    acc, zp = mono[t], 1
                    for a in range(1, f):
                        zp = O.gl_mul(zp, z)
                        acc = O.gl_add(acc, O.gl_mul(mono[t + a * m], zp))
                    h.append(acc)
                _np(out)[i, c] = O.bitreverse(np.array(h, dtype=np.uint64))

    def lde_shard_folded(self, folded, log_n, log_lde, log_shards, shard, lde):
        sp = self._shard_shift(log_n, log_lde, log_shards, shard)
        for c in range(folded.shape[0]):
            _np(lde)[c] = O.fft_natural_to_bitreversed(O.bitreverse(_np(folded)[c]), int(sp))

    def lde_shard(self, coeffs, log_n, log_lde, log_shards, shard, work, lde):
        n = 1 << log_n
        m = (n << log_lde) >> log_shards
        cosets = O.lde_cosets(log_n, log_lde)
        for c in range(coeffs.shape[0]):
            mono = O.bitreverse(_np(coeffs)[c])
            flat = np.concatenate([O.fft_natural_to_bitreversed(mono, int(s)) for s in cosets])
            _np(lde)[c] = flat[shard * m:(shard + 1) * m]

    def leaves(self, lde, out, cap_in=None, final=True, cols_before=0):
        src = _np(lde)
        if self.hasher == "blake2s":
            cin = None if cap_in is None else _np(cap_in).copy()
            _np(out)[:] = np.stack([O.blake2s_leaf_partial(None if cin is None else cin[r],
                                                           np.ascontiguousarray(src[:, r]), cols_before, final)
                                    for r in range(src.shape[1])])
            return
        if self.hasher == "keccak256":
            assert cap_in is None and final
            _np(out)[:] = np.stack([O.keccak_leaf(np.ascontiguousarray(src[:, r])) for r in range(src.shape[1])])
            return
        if cap_in is None and final:
            _np(out)[:] = np.stack([O.hash_into_leaf(np.ascontiguousarray(src[:, r])) for r in range(src.shape[1])])
            return
        # the Overwrite sponge continued from carried capacity words (sponge.rs:224-323)
        cin = None if cap_in is None else _np(cap_in).copy()
        res = np.zeros((src.shape[1], 4), dtype=np.uint64)
        for r in range(src.shape[1]):
            st = np.zeros(12, dtype=np.uint64)
            if cin is not None:
                st[8:] = cin[r]
            col = src[:, r]
            full, rem = divmod(col.shape[0], 8)
            for g in range(full):
                st[:8] = col[8 * g: 8 * g + 8]
                st = O.poseidon2_permutation(st)
            if final and rem:
                st[:8] = 0
                st[:rem] = col[8 * full:]
                st = O.poseidon2_permutation(st)
            res[r] = st[:4] if final else st[8:]
        _np(out)[:] = res

    def nodes(self, leaves, cap_size, out):
        lv = _np(leaves)
        # merkle_construct hashes leaves from elements; rebuild the node levels directly
        node = {"poseidon2": O.hash_into_node, "blake2s": O.blake2s_node, "keccak256": O.keccak_node}[self.hasher]
        cur = lv.copy()
        res = []
        while cur.shape[0] > cap_size:
            nxt = np.stack([node(cur[2 * i], cur[2 * i + 1]) for i in range(cur.shape[0] // 2)])
            res.append(nxt)
            cur = nxt
        _np(out)[:] = np.concatenate(res)
