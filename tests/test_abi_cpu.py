"""CPU: libasvrl.so and libasvrl_f32.so (the f32-operand parity build of the same sources) load
without a GPU and export every entry point include/asvrl.h declares; the ctypes structs match the
header's layout."""
import ctypes as C
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    txt = open(os.path.join(ROOT, "include", "asvrl.h")).read()
    return sorted(set(re.findall(r"\b(asvrl_[a-z0-9_]+)\s*\(", txt)))


import pytest  # noqa: E402


@pytest.mark.parametrize("ops,nbytes", [("bf16", 2), ("f32", 4)])
def test_library_exports_every_declared_symbol(ops, nbytes):
    from distributional_rl_decision_and_control_amd import _abi
    L = _abi.lib(ops)
    names = _declared()
    assert len(names) >= 9
    for n in names:
        assert hasattr(L, n), n
    assert {e[0] for e in _abi.EXPORTS} == set(names)
    assert L.asvrl_abi_version() == _abi.ABI_VERSION
    assert L.asvrl_operand_bytes() == nbytes


def test_struct_layouts():
    from distributional_rl_decision_and_control_amd import _abi
    # sizes the header implies on LP64 (checked against the compiled library's own view)
    assert C.sizeof(_abi.AsvParams) == 480
    assert C.sizeof(_abi.AsvEnvState) == 16 + 9 * 8   # ABI 17: + robot_params
    assert C.sizeof(_abi.AsvStepCtl) == 16 + 16 + 8 + 8 + 8
    assert C.sizeof(_abi.AsvStepOut) == 8 * 8
    assert C.sizeof(_abi.AsvResetCfg) == 16 + 10 * 8
    import ctypes.util  # noqa: F401
    L = _abi.lib()
    sizes = (C.c_int64 * 5)()
    L.asvrl_struct_sizes(sizes)
    assert list(sizes) == [C.sizeof(_abi.AsvParams), C.sizeof(_abi.AsvEnvState), C.sizeof(_abi.AsvStepCtl),
                           C.sizeof(_abi.AsvStepOut), C.sizeof(_abi.AsvResetCfg)]


def test_errors_are_reported_not_raised():
    from distributional_rl_decision_and_control_amd import _abi
    L = _abi.lib()
    rc = L.asvrl_c51_project(None, None, None, None, 4, 51, -1.0, 1.0, 0.04, 0.97, None, None)
    assert rc != 0
    assert b"null" in L.asvrl_last_error()


def test_fused_variant_switch_host_side():
    """asvrl_critic_fused_variant (ABI 23) is host state only: query, set, restore; anything but 4 / 8 is refused
    with a message and leaves the setting alone."""
    from distributional_rl_decision_and_control_amd import _abi
    from distributional_rl_decision_and_control_amd.fused_critic import fused_variant
    L = _abi.lib()
    default = L.asvrl_critic_fused_variant(-1)
    assert default in (4, 8)
    with fused_variant(4):
        assert L.asvrl_critic_fused_variant(-1) == 4
    assert L.asvrl_critic_fused_variant(-1) == default
    assert L.asvrl_critic_fused_variant(5) == -1
    assert b"variant" in L.asvrl_last_error()
    assert L.asvrl_critic_fused_variant(-1) == default
    with pytest.raises(_abi.AsvrlError):
        fused_variant(6)
