"""Multi-process (gloo, CPU) tests of the sharded-commit schedule that the native collective
(bj_sharded_commit_d) implements, restated in tests/sharded_model.py with the oracle's CPU
steps: column-shard ownership (contiguous, and per-chunk column runs for the column
pipeline), the coefficient all-gather order, leaf-range ownership for G <= D (whole cosets)
and G > D (sub-cosets, the fold either on the sender with an all-to-all -- the native choice
-- or on the receiver after an all-gather), an LDE at D committed over its first k < D
cosets (prover.rs:313-347: the committed block plus this rank's share of the other blocks),
the sponge carried across column chunks, subtree nodes as slices of the reference tree, and
cap assembly for cap >= G and cap < G (top levels hashed redundantly)."""
import pytest

from sharded_check import run_and_check


@pytest.mark.parametrize("world,cfg", [
    (2, (4, 5, 1, 4)),    # G == D, cap >= G
    (2, (2, 4, 2, 2)),    # G < D
    (4, (4, 4, 1, 2)),    # G > D (sub-cosets), cap < G
    (4, (8, 5, 2, 16)),   # G == D, cap > G
    (2, (32, 5, 1, 4, 1)),    # column pipeline: 4, 4, 8 columns per rank, G == D
    (4, (64, 4, 1, 2, 1)),    # column pipeline: 2, 2, 4, 8 columns per rank, G > D (sub-cosets), cap < G
    (2, (48, 4, 2, 8, 1)),    # column pipeline: 4, 4, 8, 8 columns per rank, G < D
    (2, (128, 4, 1, 4)),      # column pipeline: 4, 4, 8, 16, 32 columns per rank
    (8, (32, 4, 1, 16)),      # column pipeline: 1, 1, 2 columns per rank (first chunk 8 columns)
    (4, (4, 4, 1, 2, 0, False)),      # G > D through the all-gather of unfolded coefficients
    (4, (64, 4, 1, 2, 1, False)),     # the same, column-pipelined
    (8, (8, 4, 1, 16)),               # G = 4 D: fold by 4 on the sender, all-to-all
    (2, (48, 4, 2, 8, 1, None, "blake2s")),    # Blake2s tree, pipelined: chaining value carried
    (4, (8, 4, 1, 2, 0, None, "blake2s")),     # Blake2s tree, G > D, cap < G
    (2, (32, 4, 1, 4, 1, None, "keccak256")),  # Keccak256 tree: one chunk (no continuation)
    (2, (4, 4, 3, 4, 0, None, None, 1)),       # LDE x8, 2 cosets committed (proof.json's D / k), G == k
    (4, (16, 4, 3, 4, 1, None, None, 1)),      # the same at G = 2k (k < G <= D: fold at the receiver)
    (4, (4, 4, 2, 2, 0, None, None, 0)),       # LDE x4, one coset committed, G = D, cap < G
    (8, (8, 4, 2, 8, 0, None, None, 0)),       # G > D: sender-side fold per block, all-to-all per block
])
def test_sharded_commit_gloo(world, cfg, tmp_path):
    run_and_check(world, cfg, tmp_path, "cpu")


def test_model_rejects_bad_shapes():
    from sharded_model import ShardModel
    from shard_cpu_ops import CpuShardOps
    with pytest.raises(ValueError):
        ShardModel(3, 4, 1, 2, 0, 2, CpuShardOps())   # C % G
    with pytest.raises(ValueError):
        ShardModel(4, 4, 1, 2, 0, 3, CpuShardOps())   # G not 2^k
    with pytest.raises(ValueError):
        ShardModel(4, 1, 1, 2, 0, 8, CpuShardOps())   # G > leaves
    with pytest.raises(ValueError):
        ShardModel(4, 4, 1, 2, 0, 2, CpuShardOps(), log_k=2)   # k > D
