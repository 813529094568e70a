"""CPU-side checks of the boundary: the C-ABI library builds, loads and exports every
function include/vclip.h declares (no compute calls without a GPU); the product path
refuses CPU tensors instead of falling back."""
import ctypes

import pytest
import torch

import vclip_amd._lib as L
from vclip_amd import ops
from vclip_amd.build import LIB_PATH, build


@pytest.fixture(scope="module")
def lib():
    build()
    return L.load()


def test_header_symbols_exported(lib):
    names = L.header_functions()
    assert len(names) >= 9
    raw = ctypes.CDLL(LIB_PATH)
    for n in names:
        assert hasattr(raw, n), f"{n} declared in vclip.h but not exported"
        assert n in L.SIGNATURES, f"{n} has no ctypes signature"


def test_version_and_error_string(lib):
    assert lib.vc_version().decode().startswith("vclip")
    assert lib.vc_last_error() is not None


def test_invalid_args_fail_loudly_without_gpu(lib):
    # shape validation happens before any HIP call: a bad shape returns an error code + message
    rc = lib.vc_gemm_bf16(None, 0, None, 0, 100, 128, 64, None, 0, None, 0, None, 0, 0, 0, 0, None)
    assert rc != 0
    assert "null" in lib.vc_last_error().decode()
    rc = lib.vc_attention_fwd(ctypes.c_void_p(16), 2304, 1, 10, 12, 128, 0.1, 0, ctypes.c_void_p(16), 768, None)
    assert rc != 0 and "head_dim" in lib.vc_last_error().decode()


def test_ops_reject_cpu_tensors():
    x = torch.zeros(256, 768)
    with pytest.raises(L.VclipError):
        ops.layernorm(x, torch.ones(768), torch.zeros(768), 1e-6, torch.zeros(256, 768, dtype=torch.bfloat16))


def test_bench_cites_only_same_build_profiles(tmp_path, monkeypatch):
    """bench.py's roofline traffic / PMC numbers come from the newest profiles/ summary measured on
    THIS build (vclip_amd.build.source_hash) AND on the benchmarked workload (its "mode"): r01_v10
    beats r01_v7 (natural order), a newer summary of another build or of another mode is ignored,
    two same-build same-mode summaries that tie on their numbers cite nothing (the round-2 line
    cited TimeSformer counters for ViViT that way), and with none of this build the line says so."""
    import json as _json
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    me = bench._build_id()
    k = {"kernels": {"attn_fwd_d64_kernel": {"hbm_bytes_per_launch": 1.0}}}
    for n in ("r01_v7_traffic.json", "r01_v10_traffic.json", "r01_v9_traffic.json"):
        (prof / n).write_text(_json.dumps(dict(k, build=me, mode="fwd")))
    (prof / "r03_v1_traffic.json").write_text(_json.dumps(dict(k, build="another-build", mode="fwd")))
    (prof / "r03_v2_timesformer_traffic.json").write_text(_json.dumps(dict(k, build=me, mode="timesformer")))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench._same_build("r*_traffic.json", "fwd")[0].endswith("r01_v10_traffic.json")
    assert bench._same_build("r*_traffic.json", "timesformer")[0].endswith("r03_v2_timesformer_traffic.json")
    (prof / "r02_v1_traffic.json").write_text(_json.dumps(dict(k, build=me, mode="fwd")))
    assert bench.measured_traffic("attn_fwd_d64_kernel") == (1.0, "profiles/r02_v1_traffic.json")
    assert bench.measured_traffic(["attn_fwd_d64_kernel"] * 2) == (2.0, "profiles/r02_v1_traffic.json")
    assert bench.measured_traffic("other_kernel")[0] is None
    # a tie between two same-build same-mode files: nothing is cited
    (prof / "r02_v1_copy_traffic.json").write_text(_json.dumps(dict(k, build=me, mode="fwd")))
    v, why = bench.measured_traffic("attn_fwd_d64_kernel")
    assert v is None and why.startswith("ambiguous")
    assert bench._same_build("r*_nothing.json", "fwd")[0] is None
    for n in list(prof.iterdir()):
        if "another" not in n.read_text():
            n.unlink()
    assert bench.measured_traffic("attn_fwd_d64_kernel")[0] is None


_NO_ARGS = {"vc_version", "vc_last_error", "vc_num_cus"}


def test_every_entry_point_rejects_null_and_empty_inputs(lib):
    """Every compute entry point of include/vclip.h, called with null pointers and zero sizes, returns
    a non-zero code and sets vc_last_error (argument validation precedes any HIP call)."""
    silent = []
    for name, (argtypes, restype) in L.SIGNATURES.items():
        if name in _NO_ARGS or restype is not ctypes.c_int:
            continue
        args = []
        for t in argtypes:
            if t in (ctypes.c_float, ctypes.c_double):
                args.append(0.0)
            elif t is ctypes.c_void_p or t is ctypes.c_char_p:
                args.append(None)
            else:
                args.append(0)
        rc = getattr(lib, name)(*args)
        msg = lib.vc_last_error().decode(errors="replace")
        if rc == 0 or not msg:
            silent.append(name)
    assert not silent, f"entry points accepting null / empty input silently: {silent}"
