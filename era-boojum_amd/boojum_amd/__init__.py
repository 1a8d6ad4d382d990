"""boojum_amd -- MI355X-native witness-commitment hot path of era-boojum.

Coset LDE over Goldilocks + Poseidon2 Merkle tree with cap, as hand-written gfx950 HIP
kernels behind the C ABI in include/boojum_mi355x.h (libboojum_mi355x.so).  This
package is the host-side mirror of the reference's interface for that path:

  fft      precompute_twiddles_for_fft, fft_natural_to_bitreversed,
           ifft_natural_to_natural, distribute_powers        (src/fft/mod.rs)
  lde      transform_raw_storages_to_lde, transform_monomials_to_lde,
           ArcGenericLdeStorage, WitnessStorage             (cs/implementations/utils.rs, ...)
  merkle   MerkleTreeWithCap, Poseidon2Sponge (TreeHasher)  (cs/oracle/*)
  commit   witness_commit, CommitWorkspace                   (prover.rs:313-353)
  sharded  multi-GPU commit (one process per GPU)
"""
from ._lib import BoojumError, load  # noqa: F401
from .field import P, GENERATOR  # noqa: F401

__all__ = ["fft", "lde", "merkle", "commit", "field", "BoojumError", "load", "P", "GENERATOR"]
