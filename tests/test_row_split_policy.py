"""The heavy-row policy (dgl.kernel._split_threshold): which graphs the
default "auto" policy cuts into chunked rows. Host logic only: the chunked
kernels themselves are tested in test_gpu_kernels.py / test_accumulate.py /
test_rmat26.py."""
import pytest

from dgl import kernel


class _FakeCSR(object):
    def __init__(self, nnz, max_degree):
        self.nnz, self.max_degree = nnz, max_degree


@pytest.fixture
def policy():
    old = kernel.set_row_split("auto")
    yield kernel.set_row_split
    kernel.set_row_split(old)


def test_default_is_auto():
    assert kernel.get_row_split() == "auto" or "DGLHIP_ROW_SPLIT" in __import__("os").environ


@pytest.mark.parametrize("nnz,max_degree,expect", [
    # Reddit-shaped bench graph: the longest row is 1.35x a wave's share and
    # under the floor: one exact chain per row
    (114_848_857, 21_657, 0),
    # RMAT-26: max in-degree ~ E * 0.76^26 = 855k, 2.9x the share: chunks of
    # nnz / 12000 slots
    (1_073_741_824, 855_000, 1_073_741_824 // 12000),
    # RMAT-22 (max 160,139 measured, 8.6x the share): chunks of 5592 slots
    (67_108_864, 160_139, 67_108_864 // 12000),
    # small skewed test graphs: never split by default (bit-exact)
    (40_000, 9_000, 0),
    (2_000_000, 16_384, 0),
    (2_000_000, 16_385, 4096),
    # RMAT-26's pipelined segments at 1/8 (~30M edges, hub rows ~60k): split
    (30_000_000, 60_000, 4096),
    # a hub row that is long but not the critical path of a huge launch
    (4_000_000_000, 1_000_000, 0),
])
def test_auto_gate(policy, nnz, max_degree, expect):
    assert kernel._split_threshold(_FakeCSR(nnz, max_degree)) == expect


def test_off_and_explicit(policy):
    policy("off")
    assert kernel._split_threshold(_FakeCSR(1 << 30, 1 << 20)) == 0
    policy(1000)
    assert kernel._split_threshold(_FakeCSR(50_000, 1001)) == 1000
    assert kernel._split_threshold(_FakeCSR(50_000, 1000)) == 0


def test_policy_scales_with_the_part(policy):
    """The gate and the cut come from the part's resident waves R: a part with
    half of MI355X's (3,584) gives each wave twice the share, so rows must be
    twice as long to be the critical path and the cut is twice as long."""
    full, half = kernel._REF_WAVES, kernel._REF_WAVES // 2
    rmat26 = _FakeCSR(1_073_741_824, 855_000)
    assert kernel._split_threshold(rmat26, waves=full) == 1_073_741_824 // 12000
    assert kernel._split_threshold(rmat26, waves=half) == 1_073_741_824 // 6000
    # a 40k-slot row of a 30M-edge segment: past twice a wave's share on the
    # full part (30M / 3,584 = 8,370) but not on an eighth of it (66,964)
    seg = _FakeCSR(30_000_000, 40_000)
    assert kernel._split_threshold(seg, waves=full) == 4096
    assert kernel._split_threshold(seg, waves=full // 8) == 0
    # the Reddit-shaped bench graph stays one exact chain per row
    reddit = _FakeCSR(114_848_857, 21_657)
    assert kernel._split_threshold(reddit, waves=full) == 0
    assert kernel._split_threshold(reddit, waves=half) == 0


def test_host_parts_use_the_reference_waves():
    assert kernel._resident_waves(None) == kernel._REF_WAVES
    assert kernel._resident_waves("cpu") == kernel._REF_WAVES


@pytest.mark.gpu
def test_resident_waves_on_mi355x():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    w = kernel._resident_waves(torch.device("cuda", 0))
    props = torch.cuda.get_device_properties(0)
    assert w % props.multi_processor_count == 0
    # MI355X: 256 CUs x 7 waves per SIMD x 4 SIMDs at the kernel's 72 VGPRs
    if props.multi_processor_count == 256:
        assert w == 7168
