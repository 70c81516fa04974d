"""The pipelined device step (fleet_update_encode_device): the aggregation of one
batch and the client encode of the next in one launch must give exactly what
fleet_update_device and fleet_encode_device give as two calls -- the merged text,
merged_f32 and the next batch's uploads, byte for byte -- on the stream grid (the
fused kernel k_update_encode), on the wide tiles (k_update_tiled_encode), the flat
and woven tiles of small windows (k_update_flat, k_update_weave_encode<8 | 6>: 62,001
and 104,003 values, 20.7 k and 34.7 k groups) and on the pipelined tiles (k_update_pipe
with the encode's blocks appended). The two
separate calls are themselves checked against the oracle elsewhere
(test_gpu_parity.py, test_gpu_full_size.py)."""
import numpy as np
import pytest

import fleet_amd as F
from fleet_amd.layouts import LAYOUTS

pytestmark = pytest.mark.gpu


def _batch(codec, torch, lay, M, seed, n_values=None):
    n = lay.n_up if n_values is None else n_values
    groups = (n + 2) // 3
    hp = np.asarray(lay.header_positions(), np.int32) if n_values is None else np.zeros(0, np.int32)
    hv = lay.header_values() if n_values is None else np.zeros(0, np.float32)
    dev = torch.device("cuda", 0)
    values = torch.empty((M, 3 * groups), dtype=torch.float32, device=dev)
    codec.synth_device(seed, values, n, hp, hv)
    return n, groups, hp, values


@pytest.mark.parametrize("lay_name,M,n_values", [("synth1m", 6, None), ("synth1m", 1, None),
                                                  ("cifar10", 5, None), ("cifar100", 4, None), ("mnist", 3, None),
                                                  ("mnist", 64, None), ("synth1m", 3, 1_000_003), ("synth1m", 2, 150_001),
                                                  ("synth1m", 2, 100), ("synth1m", 4, 62_001), ("synth1m", 3, 104_003),
                                                  ("synth1m", 3, 131_075)])
def test_update_encode_equals_two_calls(codec, lay_name, M, n_values, pad=0):
    torch = pytest.importorskip("torch")
    lay = LAYOUTS[lay_name]
    n, groups, hp, values = _batch(codec, torch, lay, M, 7 + M, n_values)
    _, _, _, values_next = _batch(codec, torch, lay, M, 99 + M, n_values)
    L = F.b64_len(n)
    dev = values.device
    dampen = [1.0 / (c % 3 + 1) for c in range(M)]
    text = torch.zeros((M, 16 * groups + pad), dtype=torch.uint8, device=dev)
    codec.encode_device(values, n, text)

    # reference: the two separate calls
    merged_a = torch.zeros(16 * groups, dtype=torch.uint8, device=dev)
    f32_a = torch.zeros(3 * groups, dtype=torch.float32, device=dev)
    codec.update_device(text, L, dampen, hp, merged_a, f32_a)
    next_a = torch.zeros_like(text)
    codec.encode_device(values_next, n, next_a)
    codec.check()

    merged_b = torch.zeros_like(merged_a)
    f32_b = torch.zeros_like(f32_a)
    next_b = torch.zeros_like(text)
    codec.update_encode_device(text, L, dampen, hp, merged_b, f32_b, values_next, next_b)
    torch.cuda.synchronize()
    codec.check()
    assert torch.equal(merged_a, merged_b)
    assert torch.equal(f32_a.view(torch.int32), f32_b.view(torch.int32))
    assert torch.equal(next_a, next_b)
    assert not torch.equal(next_b, text)  # a different batch really was encoded
    print(lay_name, M, F.update_encode_kernel(L))


@pytest.mark.parametrize("lay_name,M", [("synth1m", 3), ("cifar10", 3), ("mnist", 5)])
def test_update_encode_padded_rows(codec, lay_name, M):
    """Upload rows wider than the text (pitch = 16 * groups + 48): both jobs honour the pitch."""
    test_update_encode_equals_two_calls(codec, lay_name, M, None, pad=48)


def test_update_encode_rejects_overlap_and_bad_text(codec):
    torch = pytest.importorskip("torch")
    lay = LAYOUTS["synth1m"]
    M = 2
    n, groups, hp, values = _batch(codec, torch, lay, M, 3)
    L = F.b64_len(n)
    dev = values.device
    text = torch.zeros((M, 16 * groups), dtype=torch.uint8, device=dev)
    codec.encode_device(values, n, text)
    merged = torch.zeros(16 * groups, dtype=torch.uint8, device=dev)
    with pytest.raises(F.FleetError):
        codec.update_encode_device(text, L, [1.0, 1.0], hp, merged, None, values, text)
    # an invalid Base64 char in the uploads is reported like update_device does
    nxt = torch.zeros_like(text)
    text[1, 17] = ord("*")
    codec.update_encode_device(text, L, [1.0, 1.0], hp, merged, None, values, nxt)
    torch.cuda.synchronize()
    with pytest.raises(F.FleetError):
        codec.check()


@pytest.mark.parametrize("spec,kernel", [("fused=off", " + k_encode_f32"), ("update=tiled", "k_update_tiled_encode<64>"),
                                         ("update=pipe", "k_update_pipe<16, 1, 5, 0, false> (with the encode's blocks)"),
                                         ("update=stream", "k_update_encode<256>"),
                                         ("update=stream,grid=lanes", "k_update_encode<256>"),
                                         ("update=tiled,tile=weave6", "k_update_weave_encode<6>"),
                                         ("update=tiled,tile=weave8", "k_update_weave_encode<8>"),
                                         ("update=tiled,tile=classic", "k_update_tiled_encode<64>"),
                                         ("update=tiled,tile=flat", "k_update_flat"),
                                         ("update=tiled,tile=flat,flat_w2=16", "k_update_flat"),
                                         ("update=tiled,tile=flat,tile_enc_prio=3", "k_update_flat"),
                                         ("update=tiled,tile_enc_prio=2", "k_update_tiled_encode<64>")])
def test_update_encode_under_plans(codec, plan, spec, kernel):
    """The pipelined step on each launch plan, forced on sizes the planner gives
    another kernel (fused=off: the two launches back to back)."""
    plan(spec)
    assert F.update_encode_kernel(F.b64_len(LAYOUTS["cifar10"].n_up)).endswith(kernel)
    test_update_encode_equals_two_calls(codec, "cifar10", 3, None)
    test_update_encode_equals_two_calls(codec, "synth1m", 2, 150_001)


def test_plan_overrides_are_validated():
    """fleet_set_plan rejects an unknown key or value as a whole and leaves the plan
    unchanged; the default is the empty spec."""
    F.set_plan("")
    assert F.plan() == ""
    for bad in ("update=fast", "k_update=stream", "grid", "stage_threads=0", "stage_threads=65", "fused=1",
                "update=stream,tile_mix=off", "update=tiled,tile=weave4"):
        with pytest.raises(F.FleetError):
            F.set_plan(bad)
        assert F.plan() == ""
    with F.plan_override("update=tiled; grid=plain"):
        assert F.plan() == "update=tiled,grid=plain"
        assert F.update_kernel(F.b64_len(LAYOUTS["mnist"].n_up)) == "k_update_weave<8>"
    assert F.plan() == ""
