"""CPU checks of the drop-in boundary: the in-tree C-ABI library loads and exports exactly what
include/kalibr_hip.h declares; without a GPU the product path fails loudly (no CPU fallback)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    txt = open(os.path.join(ROOT, "include", "kalibr_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(kb_[a-z_0-9]+)\s*\(", txt)))


def test_header_matches_binding_list():
    from kalibr_amd import capi
    assert _declared() == sorted(capi.EXPORTS)


def test_library_exports_every_symbol():
    from kalibr_amd import capi
    lib = capi.lib()
    for name in _declared():
        assert hasattr(lib, name), name


def test_no_cpu_fallback_without_device():
    if os.path.exists("/dev/kfd"):  # (no torch import: the product processes load only the library's HIP runtime)
        pytest.skip("GPU present")
    from kalibr_amd import capi, synth
    with pytest.raises(capi.KbError, match="no HIP device"):
        capi.Solver(synth.make_config(1, n_frames=4))


def test_product_does_not_import_oracle():
    """kalibr_amd/ (the product) must not import, link or call oracle/ (test infrastructure)."""
    for dp, _, files in os.walk(os.path.join(ROOT, "kalibr_amd")):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                src = open(os.path.join(dp, f)).read()
                assert "oracle" not in re.sub(r"(#|//).*", "", src), f
