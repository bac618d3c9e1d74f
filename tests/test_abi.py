"""The C-ABI library loads on a CPU-only host and exports every symbol include/ddm_amd.h
declares (no compute calls here)."""
import ctypes
import os
import re

from conftest import ROOT


def header_functions():
    text = open(os.path.join(ROOT, "include", "ddm_amd.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(ddm_\w+)\s*\(", text, flags=re.M)))


def test_header_lists_expected_entry_points():
    names = header_functions()
    for want in ("ddm_abi_version", "ddm_last_error", "ddm_forest_predict", "ddm_scan_streams", "ddm_mt_perms",
                 "ddm_mt_randint31", "ddm_mt_skip", "ddm_synth_block_labels", "ddm_synth_features",
                 "ddm_synth_bernoulli_streams", "ddm_rf_fit", "ddm_shuffle_generate", "ddm_shuffle_tables",
                 "ddm_shuffle_window", "ddm_shuffle_pick", "ddm_event_create"):
        assert want in names


def test_library_exports_every_declared_symbol():
    from ddm_amd import _capi
    lib = ctypes.CDLL(_capi.LIB_PATH)
    for name in header_functions():
        assert hasattr(lib, name), name
    assert set(header_functions()) == set(_capi.SIGNATURES)
    assert _capi.lib.ddm_abi_version() == _capi.ABI_VERSION


def test_struct_layouts():
    from ddm_amd import _capi, kernels
    from ddm_amd.forest import NODE_DTYPE
    assert ctypes.sizeof(_capi.DdmState) == kernels.STATE_DTYPE.itemsize == 56
    assert NODE_DTYPE.itemsize == 16
    st = kernels.fresh_states(1)[0]
    assert st["miss_prob"] == 1.0 and st["sample_count"] == 1 and st["miss_prob_sd_min"] == float("inf")


def test_invalid_args_report_errors():
    from ddm_amd import _capi
    rc = _capi.lib.ddm_mt_perms(None, None, None, 0, None, None)
    assert rc == _capi.DDM_E_ARG
    rc = _capi.lib.ddm_scan_streams(None, None, 1, None, None, None, None, 0, None, None, None, 0, None, None,
                                    None, None, None, None)
    assert rc == _capi.DDM_E_ARG
    assert b"invalid argument" in _capi.lib.ddm_last_error()
