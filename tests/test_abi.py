"""The C-ABI library loads and exports every symbol include/bppo.h declares
(no compute calls: this runs without a GPU)."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def so():
    p = os.path.join(ROOT, "burn-ppo_amd", "bppo", "libbppo.so")
    if not os.path.exists(p):
        subprocess.run(["make", "-j8", "-C", os.path.join(ROOT, "burn-ppo_amd")], check=True)
    return p


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "bppo.h")).read()
    return sorted(set(re.findall(r"\b(bppo_[a-z_0-9]+)\s*\(", txt)))


def test_header_declares_expected_surface():
    syms = header_symbols()
    import bppo._lib as L
    assert sorted(L.EXPORTS) == syms


def test_library_exports_every_header_symbol(so):
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (bppo_[a-z_0-9]+)$", out, re.M))
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, missing


def test_library_loads_and_reports_version(so):
    import bppo._lib as L
    lib = L.lib()
    assert lib.bppo_version().decode().startswith("bppo-mi355x")


def test_offload_arch_is_gfx950(so):
    # the embedded clang offload bundle names its targets (no extraction to disk)
    data = open(so, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in data


def test_host_libm_path_without_gpu():
    import numpy as np
    import bppo._lib as L
    x = np.linspace(1e-6, 1.0, 1000, dtype=np.float32)
    y = np.zeros_like(x)
    assert L.lib().bppo_debug_libm(0, 0, x.ctypes.data, y.ctypes.data, x.size) == 0
    assert np.allclose(y, np.log(x), rtol=1e-6, atol=1e-7)


# ------------------------------------------------------------ struct layouts ---
_C_TYPES = {"int32_t": ("i32", C.c_int32), "float": ("f32", C.c_float), "double": ("f64", C.c_double),
            "uint64_t": ("u64", C.c_uint64)}
_CONSTS = {"BPPO_MAX_PLAYERS": 6}


def _header_struct(name):
    """[(field, type, array_len or 0)] of `typedef struct { ... } name;` in include/bppo.h"""
    txt = open(os.path.join(ROOT, "include", "bppo.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    body = re.search(r"typedef struct \{([^}]*)\}\s*%s;" % name, txt).group(1)
    out = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        ty, rest = decl.split(None, 1)
        for f in rest.split(","):
            m = re.fullmatch(r"\s*(\w+)\s*(?:\[(\w+)\])?\s*", f)
            n = 0 if m.group(2) is None else int(_CONSTS.get(m.group(2), m.group(2)))
            out.append((m.group(1), _C_TYPES[ty][0], n))
    return out


def _ctypes_struct(cls):
    inv = {v[1]: v[0] for v in _C_TYPES.values()}
    out = []
    for f, t in cls._fields_:
        if hasattr(t, "_length_"):
            out.append((f, inv[t._type_], t._length_))
        else:
            out.append((f, inv[t], 0))
    return out


def _rust_struct(name):
    txt = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    i = txt.index("pub struct %s {" % name) + len("pub struct %s {" % name)
    body = re.sub(r"//[^\n]*", "", txt[i:txt.index("}", i)])
    out = []
    for m in re.finditer(r"pub (\w+):\s*(\[\s*(\w+)\s*;\s*(\d+)\s*\]|\w+)", body):
        if m.group(3):
            out.append((m.group(1), m.group(3), int(m.group(4))))
        else:
            out.append((m.group(1), m.group(2), 0))
    return out


@pytest.mark.parametrize("c_name,rust_name,attr", [
    ("bppo_config", "BppoConfig", "Config"), ("bppo_update_metrics", "BppoUpdateMetrics", "UpdateMetrics"),
    ("bppo_episode", "BppoEpisode", "Episode"), ("bppo_rollout_info", "BppoRolloutInfo", "RolloutInfo")])
def test_struct_layouts_match_header(so, c_name, rust_name, attr):
    """include/bppo.h, the ctypes binding (bppo/_lib.py) and the Rust binding in
    INTEGRATION.md list the same fields, in the same order, with the same types; and the
    library's sizeof exports equal the ctypes sizes."""
    import bppo._lib as L
    hdr = _header_struct(c_name)
    assert _ctypes_struct(getattr(L, attr)) == hdr
    assert _rust_struct(rust_name) == hdr
    size_fn = {"bppo_config": "bppo_config_size", "bppo_update_metrics": "bppo_update_metrics_size",
               "bppo_episode": "bppo_episode_size", "bppo_rollout_info": "bppo_rollout_info_size"}[c_name]
    assert getattr(L.lib(), size_fn)() == C.sizeof(getattr(L, attr))


@pytest.mark.parametrize("preset,over", [
    ("cartpole", dict(split_networks=True, num_hidden=8)),                         # 2 * 8 + 2 = 18 layers
    ("connect_four", dict(hidden_size=32, num_hidden=15)),                         # 17
    ("liars_dice_ctde", dict(num_hidden=8, critic_num_hidden=7)),                  # 17
    ("connect_four", dict(network_type="cnn", split_networks=True, num_conv_layers=4,
                          conv_channels=[4], cnn_num_fc_layers=4))])               # 2 * 8 + 2 = 18
def test_create_rejects_nets_over_16_layers_before_any_hip_call(so, preset, over):
    """NetLayout holds 16 layers; deeper nets (any net type) are refused with
    BPPO_ERR_UNSUPPORTED by bppo_create's configuration check, which runs before the
    first HIP call (so this runs without a GPU)."""
    import bppo
    import bppo._lib as L
    from bppo.host import to_struct
    cfg = bppo.make_config(preset, num_envs=8, num_steps=4, **over)
    s = to_struct(cfg)
    h = C.c_void_p()
    st = L.lib().bppo_create(C.byref(s), 0, None, C.byref(h))
    try:
        assert st == L.ERR_UNSUPPORTED, (st, L.lib().bppo_last_error(h))
        assert b"16 layers" in L.lib().bppo_last_error(h)
    finally:
        L.lib().bppo_destroy(h)


def test_null_context_is_an_argument_error(so):
    """every setter checks its context before touching it (bppo_optimizer_set
    dereferenced a NULL ctx); no HIP call is made, so this runs without a GPU."""
    import bppo._lib as L
    lib = L.lib()
    buf = (C.c_float * 4)()
    steps = (C.c_int32 * 4)()
    assert lib.bppo_optimizer_set(None, buf, buf, steps, 4) == L.ERR_ARG
    assert lib.bppo_optimizer_get(None, buf, buf, steps, 4) == L.ERR_ARG
    assert lib.bppo_params_set(None, buf, 4) == L.ERR_ARG
    assert lib.bppo_rng_set(None, 0) == L.ERR_ARG
    assert lib.bppo_set_explained_variance_mode(None, 1) == L.ERR_ARG
    assert lib.bppo_set_minibatch_kernel(None, 2) == L.ERR_ARG
