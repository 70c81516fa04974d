"""The C-ABI library without a GPU: it loads, exports every symbol declared in
include/fleet_codec.h, its host-only helpers work, and compute entry points
fail loudly (no CPU fallback exists)."""
import ctypes as C

import numpy as np
import pytest

import fleet_amd as F
from fleet_amd.layouts import CIFAR10, CIFAR100, LAYOUTS, MNIST


def test_library_exports_every_declared_symbol():
    L = F.lib()
    declared = F.exported_symbols_from_header()
    assert len(declared) >= 25
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    assert F.lib().fleet_version().startswith(b"fleet-mi355x")


def test_b64_lengths():
    for n in list(range(0, 50)) + [22961, 313867, 1 << 20]:
        L = F.lib().fleet_b64_len(n)
        assert L == 4 * ((4 * n + 2) // 3) == F.b64_len(n)
        assert F.lib().fleet_b64_count(L) == n


@pytest.mark.parametrize("lay", [MNIST, CIFAR10, CIFAR100, LAYOUTS["synth1m"]])
def test_layout_from_sizes(lay):
    pos, n_up = F.layout_from_sizes(lay.w_sizes, lay.b_sizes)
    assert n_up == lay.n_up
    assert pos.tolist() == lay.header_positions()


def test_layout_matches_oracle_mask(oracle):
    for lay in (MNIST, CIFAR10):
        mask = oracle.header_mask(list(lay.w_sizes), list(lay.b_sizes))
        assert np.nonzero(mask)[0].tolist() == lay.header_positions()


def test_no_cpu_fallback_without_gpu():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    with pytest.raises(F.FleetError) as e:
        F.Codec(0)
    assert e.value.code == F.FLEET_ERR_HIP
    h = C.c_void_p()
    assert F.lib().fleet_create(0, C.byref(h)) == F.FLEET_ERR_HIP


def test_null_context_rejected():
    L = F.lib()
    n = C.c_size_t(0)
    assert L.fleet_encode_f32(None, None, 0, None, 0, C.byref(n)) == F.FLEET_ERR_ARG
    assert L.fleet_update(None, None, None, 0, None, None, 0, None, None) == F.FLEET_ERR_ARG
    assert L.fleet_update_device(None, None, 0, 0, 0, None, None, 0, 0, 0, None, None, None) == F.FLEET_ERR_ARG
    assert L.fleet_update_encode_device(None, None, 0, 0, 0, None, None, 0, None, None, None, 0, None,
                                        None) == F.FLEET_ERR_ARG


def test_plan_overrides_validated_on_host():
    """fleet_set_plan is host-only: a spec with an unknown key or value is rejected
    as a whole (the plan stays as it was), a valid one is normalised, "" restores
    the default. No environment variable other than FLEET_EXPERIMENTS (read once)
    reaches the launch path (kernels.hip reads no other)."""
    import os
    F.set_plan("")
    for bad in ("update=fast", "k_update=stream", "grid", "stage_pieces=0", "fused=1", "update=stream,tile_mix=off",
                "update=tiled,tile=weave3", "update=stream,stream_enc=inline", "update=tiled,weave_enc=inline"):
        with pytest.raises(F.FleetError):
            F.set_plan(bad)
        assert F.plan() == ""
    F.set_plan(" update=pipe ;fused=off,stage_threads=3")
    assert F.plan() == "update=pipe,fused=off,stage_threads=3"
    F.set_plan("")
    assert F.plan() == ""
    src = open(os.path.join(F.ROOT, "fleet_amd", "csrc", "kernels.hip")).read()
    assert src.count("getenv(") == 1 and 'getenv("FLEET_EXPERIMENTS")' in src
    assert "getenv(" not in open(os.path.join(F.ROOT, "fleet_amd", "csrc", "fleet_codec.cpp")).read()


GRID_SIZES = [1, 2, 16, 17, 83, 84, 85, 255, 256, 257, 6_667, 7_654, 16_668, 32_768, 50_001, 65_537, 100_001,
              104_623, 110_413, 131_072, 174_763, 349_526, 1_398_102]


# The default launch plan per size (DESIGN.md §4 "Launch choice", kernels.hip plan_update),
# planned for 256 CUs (the host has no device: device_simds' fallback). (groups, update
# alone, fused step) at the ends of every range.
DEFAULT_PLAN = [
    (1_000, "k_update_pipe<16, 1, 5, 0, false>", "k_update_pipe<16, 1, 5, 0, false> (with the encode's blocks)"),
    (14 * 1024 - 1, "k_update_pipe<16, 1, 5, 0, false>", "k_update_pipe<16, 1, 5, 0, false> (with the encode's blocks)"),
    (14 * 1024, "k_update_pipe<16, 1, 5, 0, false>", "k_update_weave_encode<8>"),
    (24 * 1024 - 1, "k_update_pipe<16, 1, 5, 0, false>", "k_update_weave_encode<8>"),
    (24 * 1024, "k_update_weave<8>", "k_update_weave_encode<8>"),
    (32 * 1024, "k_update_weave<8>", "k_update_weave_encode<6>"),
    (40 * 1024 - 1, "k_update_weave<8>", "k_update_weave_encode<6>"),
    (40 * 1024, "k_update_weave<8>", "k_update_flat"),
    (3 * 64 * 256, "k_update_weave<8>", "k_update_flat"),
    (3 * 64 * 256 + 1, "k_update_flat", "k_update_flat"),
    (65_535, "k_update_flat", "k_update_flat"),
    (65_536, "k_update_flat", "k_update_tiled_encode<64>"),
    (131_071, "k_update_flat", "k_update_tiled_encode<64>"),
    (131_072, "k_update_mixed<256, false>", "k_update_encode<256>"),
    (349_526, "k_update_mixed<256, false>", "k_update_encode<256>"),
]


@pytest.mark.parametrize("groups,upd,fused", DEFAULT_PLAN)
def test_default_plan_table(groups, upd, fused):
    """Every remaining kernel form is the default at some size, in the ranges DESIGN.md
    §4 lists."""
    F.set_plan("")
    assert F.update_kernel(16 * groups) == upd
    assert F.update_encode_kernel(16 * groups) == fused


@pytest.mark.parametrize("spec", ["", "update=stream", "update=stream,grid=plain", "update=stream,grid=lanes",
                                  "update=tiled", "update=tiled,tile=classic", "update=pipe",
                                  "update=tiled,tile=weave6", "update=tiled,tile=weave8", "update=tiled,tile=flat",
                                  "update=tiled,tile=flat,flat_w2=16",
                                  "update=tiled,tile=flat,flat_w2=64", "update=tiled,tile=flat,flat_w2=21"])
def test_launch_grid_covers_every_group(spec):
    """The aggregation's grid (fleet_update_plan_grid) covers every group of the
    bucket exactly once and launches no block past it, under every plan: the stream
    grid's group-per-lane blocks (256 groups) then value-per-lane blocks (84 groups:
    4 waves x 21), the tiles' two widths, the pipelined 16-group tiles. (An r04 plan
    change once dropped the stream grid's last ragged block when the plain grid
    covered the bucket; found on the GPU, pinned here on the host.)"""
    F.set_plan(spec)
    try:
        for groups in GRID_SIZES:
            g = F.update_plan_grid(16 * groups)
            b = g["blocks"]
            if g["kind"] == "stream":
                covered_a = 256 * g["n_a"]
                if covered_a >= groups:
                    assert b == g["n_a"] and 256 * (b - 1) < groups, (groups, g)
                else:
                    rest = groups - covered_a
                    assert b - g["n_a"] == -(-rest // 84), (groups, g)
            elif g["kind"] == "tiled":  # one width (tile=classic: the fused step's tiles alone)
                assert g["n_w"] < 0 and b == -(-groups // 64), (groups, g)
            elif g["kind"] == "weave":
                assert b == -(-groups // 64), (groups, g)
            elif g["kind"] == "flat":  # n_w 64-group tiles, then n_n tiles of 2^n_a groups, the last ragged
                w2 = g["n_a"]
                assert b == g["n_w"] + g["n_n"] and 1 <= w2 <= 64, (groups, g)
                cov = 64 * g["n_w"] + w2 * g["n_n"]
                assert cov >= groups and (g["n_n"] == 0 or cov - w2 < groups), (groups, g)
                assert 64 * g["n_w"] <= groups, (groups, g)
                if "flat_w2=" in spec:
                    assert w2 == int(spec.split("flat_w2=")[1]), (groups, g)
            else:
                assert b == -(-groups // 16), (groups, g)
            if spec.startswith("update="):
                want = spec.split(",")[0].split("=")[1]
                if want == "tiled" and "tile=classic" not in spec:  # the update alone: flat tiles unless asked,
                    # the woven 8-wave tiles up to three per CU (256 CUs without a device)
                    want = ("weave" if "tile=weave" in spec or ("tile=" not in spec and groups <= 3 * 64 * 256)
                            else "flat")
                assert g["kind"] == want, (spec, g)
    finally:
        F.set_plan("")


def test_no_cuda_compat_layers_in_the_product():
    """The product sources use AMD's own libraries directly: no hipCUB (the CUB-compatible
    layer; the model codec's sort and scans are rocPRIM), no CUDA headers or dual paths."""
    import glob
    import os
    for path in glob.glob(os.path.join(F.ROOT, "fleet_amd", "csrc", "*")):
        src = open(path).read()
        assert "hipcub" not in src, path
        assert "cuda_runtime" not in src and "__CUDACC__" not in src and "__HIP_PLATFORM_AMD__" not in src, path
