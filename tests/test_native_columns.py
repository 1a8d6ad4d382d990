"""Host logic of the native collective commit (no GPU): bj_sharded_columns deals the trace
columns exactly as the CPU model of its schedule (tests/sharded_model.py, which the gloo tests
check against the oracle) does, and rejects the shapes the reference's asserts reject."""
import pytest

from boojum_amd._lib import BoojumError
from boojum_amd.sharded import native_columns
from sharded_model import ShardModel
from shard_cpu_ops import CpuShardOps


@pytest.mark.parametrize("n_cols", [8, 16, 24, 32, 48, 64, 96, 128, 256])
@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("hasher", ["poseidon2", "blake2s", "keccak256"])
def test_native_deal_matches_python_orchestration(n_cols, world, hasher):
    seen = []
    for rank in range(world):
        ws = ShardModel(n_cols, 4, 1, 2, rank, world, CpuShardOps(hasher), hasher=hasher)
        cols = native_columns(n_cols, world, rank, hasher)
        assert cols == ws.my_columns, (n_cols, world, rank, hasher)
        seen += cols
    assert sorted(seen) == list(range(n_cols))


def test_native_deal_single_rank_is_identity():
    assert native_columns(256, 1, 0) == list(range(256))
    assert native_columns(93, 1, 0, "blake2s") == list(range(93))


def test_native_deal_c3_at_eight_ranks():
    """C3 at G = 8: chunks of 1, 1, 2, 4, 8, 16 columns per rank (the first chunk 8 columns)."""
    cols = native_columns(256, 8, 3)
    assert cols[:2] == [3, 11] and cols[2:4] == [22, 23] and len(cols) == 32


def test_native_deal_rejects_bad_shapes():
    with pytest.raises(BoojumError):
        native_columns(12, 8, 0)      # C % G
    with pytest.raises(BoojumError):
        native_columns(16, 4, 4)      # rank >= G
