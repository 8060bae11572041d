"""Hand-written LSD radix sort (csrc/sort_hip.hip) vs a stable torch sort of the same bits.

Covers partial tiles, sizes below one wave, bit ranges that are not a multiple of the digit
width, a constant digit (every key in one bucket of a pass), the INT64_MAX hole sentinel of the
keyed-state passes, and stability (equal keys keep their input order: values are the input
positions)."""
import pytest
import torch

from mxstream.ops import kernels as K
from mxstream.ops.native import load

pytestmark = pytest.mark.gpu


def _ref(keys: torch.Tensor, vals: torch.Tensor, bits: int):
    k = keys if bits == 64 else keys & ((1 << bits) - 1)
    ks = k ^ K.I64_MIN if bits == 64 else k
    order = torch.sort(ks.cpu(), stable=True).indices
    return keys.cpu()[order], vals.cpu()[order]


@pytest.mark.parametrize("n", [1, 37, 64, 4095, 4096, 4097, 100_003, 1 << 20])
@pytest.mark.parametrize("bits", [5, 8, 13, 35, 64])
def test_sort_pairs_matches_stable_sort(gpu_device, n, bits):
    g = torch.Generator().manual_seed(n * 131 + bits)
    hi = (1 << min(bits, 62))
    keys = torch.randint(0, hi, (n,), generator=g, dtype=torch.int64)
    if bits == 64:
        keys = keys * 3 - (1 << 62)  # negative patterns too (unsigned order of the bits)
    vals = torch.arange(n, dtype=torch.int64)
    ko, vo = K.sort_pairs(keys.to(gpu_device), vals.to(gpu_device), bits=bits)
    ek, ev = _ref(keys, vals, bits)
    assert torch.equal(ko.cpu(), ek)
    assert torch.equal(vo.cpu(), ev)


def test_sort_pairs_few_distinct_and_sentinels(gpu_device):
    """Slot-major keys as the rolling pass builds them (slot << shift | arrival) with a few hot
    slots, holes as INT64_MAX (sorted last over the used bits), and a sort over a bit range that
    starts above bit 0 (the direct rolling path sorts the slot bits only)."""
    n = 300_000
    g = torch.Generator().manual_seed(5)
    slot = torch.randint(0, 7, (n,), generator=g, dtype=torch.int64) * 1000
    shift = 19
    keys = (slot << shift) | torch.arange(n, dtype=torch.int64)
    keys[::101] = K.I64_MAX
    vals = torch.randint(-(1 << 60), 1 << 60, (n,), generator=g, dtype=torch.int64)
    nbits = shift + 14
    m = load()
    dev = gpu_device
    kin, vin = keys.to(dev), vals.to(dev)
    ko, vo = torch.empty_like(kin), torch.empty_like(vin)
    need = m.gpu_sort_pairs_temp_bytes(n, shift, nbits)
    tmp = torch.empty(need, dtype=torch.uint8, device=dev)
    m.gpu_sort_pairs(tmp.data_ptr(), need, kin.data_ptr(), ko.data_ptr(), vin.data_ptr(),
                     vo.data_ptr(), n, shift, nbits, torch.cuda.current_stream(dev).cuda_stream)
    sel = (keys >> shift) & ((1 << (nbits - shift)) - 1)
    order = torch.sort(sel, stable=True).indices
    assert torch.equal(ko.cpu(), keys[order])
    assert torch.equal(vo.cpu(), vals[order])
    assert torch.equal(kin.cpu(), keys)  # the input is never written
