"""The C ABI library builds/loads and exports every entry point include/maleague.h declares (CPU only:
no compute call is made without a GPU)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "maleague.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mlg_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for need in ["mlg_rollout", "mlg_env_reset", "mlg_env_step", "mlg_env_observe", "mlg_agent_forward",
                 "mlg_mac_forward", "mlg_select_actions", "mlg_pack_agent", "mlg_qmix_forward", "mlg_last_error"]:
        assert need in syms


def test_library_exports_every_declared_symbol():
    from maleague import _native
    lib = _native.load()
    nm = subprocess.run(["nm", "-D", "--defined-only", _native.lib_path()], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (mlg_[a-z0-9_]+)", nm))
    for s in declared_symbols():
        assert s in exported, f"{s} declared in maleague.h but not exported"
        assert hasattr(lib, s)
    assert set(_native.SIGNATURES) >= set(declared_symbols())
    assert lib.mlg_version().decode().startswith("maleague-gfx950")


def test_library_is_gfx950_code_object():
    from maleague import _native
    blob = open(_native.lib_path(), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob, "libmaleague.so must embed a gfx950 code object"


def test_calls_fail_loudly_without_gpu():
    import torch
    from maleague import _native
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_native.NativeError):
        _native.call("mlg_env_reset", None, None, None)


def test_argument_validation_messages():
    """Host-side checks run before any launch: bad specs are rejected with a message."""
    from maleague import _native
    from maleague.envs.teams_env import TeamsEnvSpec
    lib = _native.load()
    spec = TeamsEnvSpec.from_env_args({"match_build_plan": "small"}).to_c()
    spec.n_actions = 3
    st = _native.MlgEnvState()
    rc = lib.mlg_env_reset(_native.byref(spec), _native.byref(st), None)
    assert rc != 0 and b"n_actions" in lib.mlg_last_error()
