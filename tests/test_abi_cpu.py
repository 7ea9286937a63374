"""CPU-side checks of the C-ABI library (no GPU compute): it loads, exports
every entry point include/rcbf_hip.h declares, and the ctypes mirror of
rcbf_params has the compiled size; plus host-side argument validation."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "rcbf_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|const char\*)\s+(rcbf_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_path_entry_points():
    fns = header_functions()
    for f in ("rcbf_build", "rcbf_qp_solve", "rcbf_safe_action", "rcbf_safe_action_backward",
              "rcbf_env_step", "rcbf_safe_step", "rcbf_cascade_u_safe", "rcbf_env_reset", "rcbf_safe_rollout"):
        assert f in fns


def test_library_exports_every_declared_symbol():
    from rcbf_amd import _lib
    lib = _lib.load()
    for f in header_functions():
        assert hasattr(lib, f), f
        assert f in _lib.SIGNATURES, f"ctypes binding missing for {f}"


def test_params_struct_size_and_abi():
    from rcbf_amd import _lib
    lib = _lib.load()
    assert lib.rcbf_abi_version() == _lib.ABI_VERSION
    assert lib.rcbf_params_size() == ctypes.sizeof(_lib.RcbfParams)
    assert b"gfx950" in lib.rcbf_version()


def test_argument_validation_without_gpu():
    """Bad arguments are rejected on the host before any launch."""
    from rcbf_amd import _lib
    lib = _lib.load()
    p = _lib.RcbfParams()
    p.mode = 7
    assert lib.rcbf_safe_action(ctypes.byref(p), 4, None, None, None, None, None, None, None, None) == 1001
    p.mode = _lib.MODE_UNICYCLE
    p.num_hazards = 0
    assert lib.rcbf_safe_action(ctypes.byref(p), 4, None, None, None, None, None, None, None, None) == 1002
    p.num_hazards = 3
    assert lib.rcbf_safe_action(ctypes.byref(p), 4, None, None, None, None, None, None, None, None) == 1003
    assert lib.rcbf_safe_action(ctypes.byref(p), -1, None, None, None, None, None, None, None, None) == 1002
    # empty batch is a no-op
    assert lib.rcbf_safe_action(ctypes.byref(p), 0, None, None, None, None, None, None, None, None) == 0
    assert lib.rcbf_qp_solve(ctypes.byref(p), 4, 4, 4, None, None, None, None, 1, None, None, None, None, None) == 1002
    assert lib.rcbf_qp_solve_f64(ctypes.byref(p), 4, 2, 17, None, None, None, None, 1, None, None, None, None,
                                 None) == 1002
    assert lib.rcbf_qp_solve_f64(ctypes.byref(p), 4, 2, 4, None, None, None, None, 1, None, None, None, None,
                                 None) == 1003
    # rcbf_qp_backward: n in 1..3, m in 1..16, P/G/h/grad_z required, every gradient output optional
    assert lib.rcbf_qp_backward(ctypes.byref(p), 4, 0, 4, None, None, None, None, 1, None, None, None, None, None,
                                None) == 1002
    assert lib.rcbf_qp_backward(ctypes.byref(p), 4, 3, 7, None, None, None, None, 1, None, None, None, None, None,
                                None) == 1003
    assert lib.rcbf_qp_backward(ctypes.byref(p), 0, 3, 7, None, None, None, None, 1, None, None, None, None, None,
                                None) == 0
    # the saved-solution pair: the forward requires the z64 buffer; the backward takes it nullable (re-solves)
    assert lib.rcbf_qp_solve_saved(ctypes.byref(p), 4, 3, 7, None, None, None, None, 1, None, None, None, None,
                                   None) == 1003
    assert lib.rcbf_qp_backward_saved(ctypes.byref(p), 4, 4, 7, None, None, None, None, 1, None, None, None, None,
                                      None, None, None) == 1002
    assert lib.rcbf_qp_backward_saved(ctypes.byref(p), 4, 3, 7, None, None, None, None, 1, None, None, None, None,
                                      None, None, None) == 1003


def test_params_from_env_attributes():
    from rcbf_amd import _lib
    from rcbf_amd.envs import _EnvSpec
    from rcbf_amd.params import make_params
    spec = _EnvSpec("Unicycle")
    p = make_params(spec, 40.0, k_d=3.0, l_p=0.05)
    assert p.mode == _lib.MODE_UNICYCLE and p.num_hazards == 5
    assert p.hazards_xy[2] == -1.5 and p.hazards_xy[3] == 1.5 and p.hazards_radius == 0.6
    assert p.u_min[0] == -2.5 and p.u_max[1] == 2.5 and p.l_p == 0.05 and p.k_d == 3.0
    spec = _EnvSpec("SimulatedCars")
    p = make_params(spec, 20.0)
    assert p.mode == _lib.MODE_SIMULATED_CARS and p.kp == 4.0 and p.k_brake == 20.0
    assert p.u_min[0] == -10.0 and p.u_max[0] == 10.0

    class Bad:
        dynamics_mode = "SafetyGym"

    with pytest.raises(Exception, match="Dynamics mode not supported."):
        make_params(Bad(), 1.0)


def test_layer_requires_device():
    """No silent CPU fallback: without a HIP device the product path raises."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    from rcbf_amd.envs import BatchedSimulatedCarsEnv
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        BatchedSimulatedCarsEnv(4)


def test_state_pair_layout_roundtrip():
    """envs.pairs_to_rows / rows_to_pairs restate the device layout of
    include/rcbf_hip.h: pair p of env i at x[2(pB+i)+j], odd last component
    at x[(n_s-1)B+i]."""
    import torch
    from rcbf_amd.envs import pairs_to_rows, rows_to_pairs
    for n_s, B in [(10, 7), (3, 5), (3, 1), (10, 1), (4, 64)]:
        rows = torch.arange(B * n_s, dtype=torch.float64).reshape(B, n_s)
        xf = rows_to_pairs(rows)
        assert xf.shape == (n_s * B,)
        for i in range(B):
            for k in range(n_s):
                if k < 2 * (n_s // 2):
                    idx = 2 * ((k // 2) * B + i) + (k % 2)
                else:
                    idx = (n_s - 1) * B + i
                assert xf[idx] == rows[i, k]
        assert torch.equal(pairs_to_rows(xf, n_s, B), rows)
        if B == 1:
            assert torch.equal(xf, rows[0])


def test_cascade_get_cbfs_and_min_h():
    """CascadeCBFLayer.get_cbfs / get_min_h_val (cbf_qp.py:288-358): host
    numpy helpers, radius + 0.07 buffer, look-ahead output for the unicycle."""
    import numpy as np
    from rcbf_amd.cbf_qp import CascadeCBFLayer
    from rcbf_amd.envs import _EnvSpec
    env = _EnvSpec("Unicycle")
    cl = CascadeCBFLayer(env, l_p=0.03)
    get_h, get_dhdx = cl.get_cbfs(env.hazards_locations, env.hazards_radius)
    s = np.array([0.5, -0.2, 0.7])
    p = np.array([s[0] + 0.03 * np.cos(s[2]), s[1] + 0.03 * np.sin(s[2])])
    hz = np.asarray(env.hazards_locations)
    assert np.allclose(get_h(s), 0.5 * (((p - hz) ** 2).sum(1) - 0.67 ** 2), rtol=0, atol=1e-15)
    assert np.allclose(get_dhdx(s), p - hz, rtol=0, atol=1e-15)
    assert cl.get_min_h_val(s) == np.min(get_h(s))
    centre = np.array([hz[0, 0] - 0.03, hz[0, 1], 0.0])
    assert abs(cl.get_min_h_val(centre) + 0.5 * 0.67 ** 2) < 1e-12


def test_fast_binding_loads_and_validates():
    """The CPython binding of rcbf_safe_step (csrc/rcbf_pyfast.cpp) is built
    next to librcbf_hip.so and forwards to the same C-ABI (argument checks run
    before any launch, so this needs no GPU)."""
    from rcbf_amd import _lib, _rcbf_fast
    _lib.load()
    p = _lib.RcbfParams()
    p.mode = _lib.MODE_SIMULATED_CARS
    a = ctypes.addressof(p)
    assert _rcbf_fast.safe_step(a, 0, *([0] * 19)) == 0          # empty batch: no-op
    assert _rcbf_fast.safe_step(a, 4, *([0] * 19)) == 1003       # NULL buffers
    p.mode = 9
    assert _rcbf_fast.safe_step(a, 4, *([0] * 19)) == 1001       # bad mode
    with pytest.raises(TypeError):
        _rcbf_fast.safe_step(a, 4)
    p.mode = _lib.MODE_SIMULATED_CARS
    assert _rcbf_fast.safe_step_seq(a, 4, 3, 0, 0, 0, 0, [0], *([0] * 14)) == 1003  # NULL u_rl pointer
    assert _rcbf_fast.safe_step_seq(a, 0, 3, 0, 0, 0, 0, [0], *([0] * 14)) == 0     # empty batch
    assert _rcbf_fast.env_step_sync(a, 1, *([0] * 11)) == 1003                      # NULL host block
    with pytest.raises(ValueError):
        _rcbf_fast.safe_step_seq(a, 4, 3, 0, 0, 0, 0, [], *([0] * 14))


def test_fast_binding_follows_the_library_override(tmp_path):
    """With RCBF_HIP_LIB pointing at another copy of the library, the CPython
    binding calls into THAT copy (the one ctypes loaded), not a second,
    default copy (variant benches must measure the variant)."""
    import shutil
    import subprocess
    import sys
    from rcbf_amd import _lib
    variant = tmp_path / "librcbf_variant.so"
    shutil.copy(_lib.LIB_PATH, variant)
    code = (
        "import ctypes, sys\n"
        f"sys.path[:0] = [{os.path.join(ROOT, 'sac-rcbf_amd')!r}]\n"
        "from rcbf_amd import _lib\n"
        "lib = _lib.load()\n"
        "got = _lib.fast().bound()\n"
        "want = tuple(_lib.entry_address(lib, n) for n in _lib.FAST_ENTRY_POINTS)\n"
        "assert got == want, (got, want)\n"
        "maps = [l.split() for l in open('/proc/self/maps') if l.rstrip().endswith('librcbf_variant.so')]\n"
        "spans = [tuple(int(v, 16) for v in m[0].split('-')) for m in maps]\n"
        "assert all(any(lo <= a < hi for lo, hi in spans) for a in got), 'binding points outside the variant'\n"
        "assert not any(l.rstrip().endswith('/librcbf_hip.so') for l in open('/proc/self/maps'))\n"
        "print('ok')\n")
    env = dict(os.environ, RCBF_HIP_LIB=str(variant))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


def _header_struct_fields(name):
    """Field names of `typedef struct name { ... } name;` in include/rcbf_hip.h, in order."""
    import re
    src = open(os.path.join(ROOT, "include", "rcbf_hip.h")).read()
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), src, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = []
    for decl in (d.strip() for d in body.split(";") if d.strip()):  # "double kp, k_brake" declares two
        first, *more = decl.split(",")
        names.append(re.match(r"[\w\s\*]+?[\s\*](\w+)\s*(\[.*\])?$", first.strip()).group(1))
        names += [re.match(r"\**\s*(\w+)", m.strip()).group(1) for m in more]
    return names


@pytest.mark.parametrize("cname,pyname", [("rcbf_params", "RcbfParams"), ("rcbf_gp_model", "RcbfGpModel")])
def test_ctypes_mirrors_follow_the_header(cname, pyname):
    """The ctypes mirrors in rcbf_amd._lib name the header's fields in the
    header's order (e.g. rcbf_gp_model.flags, which carries RCBF_GP_RT_UPPER)."""
    from rcbf_amd import _lib
    assert [f[0] for f in getattr(_lib, pyname)._fields_] == _header_struct_fields(cname)
    assert _lib.GP_RT_UPPER == 1


def test_header_constants_match_the_python_mirror():
    """Every #define the Python side mirrors has the header's value (e.g. the
    Jacobian's "no gradient" marker, RCBF_JAC_NO_GRAD, a NaN payload that
    rcbf_safe_action_apply_jac tells apart from a NaN of the solve)."""
    import re
    from rcbf_amd import _lib
    src = open(os.path.join(ROOT, "include", "rcbf_hip.h")).read()
    defs = {k: int(v.rstrip("ULul"), 0) for k, v in re.findall(r"#define\s+(RCBF_\w+)\s+(0x[0-9A-Fa-f]+U?L*|\d+)\b", src)}
    assert defs["RCBF_GP_RT_UPPER"] == _lib.GP_RT_UPPER
    assert defs["RCBF_JAC_NO_GRAD"] == _lib.JAC_NO_GRAD
    import struct
    v = struct.unpack("<d", struct.pack("<Q", _lib.JAC_NO_GRAD))[0]
    assert v != v and _lib.JAC_NO_GRAD != 0x7FF8000000000000  # a NaN, not the canonical one


def _steps_code_object_kernels():
    """AMDGPU metadata of librcbf_steps.co (the code object the AQL path
    loads; built by __graft_entry__.build from rcbf_env.o)."""
    import subprocess

    import yaml
    co = os.path.join(ROOT, "sac-rcbf_amd", "rcbf_amd", "librcbf_steps.co")
    if not os.path.exists(co):
        pytest.skip("librcbf_steps.co not built")
    txt = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", co], check=True, capture_output=True,
                         text=True).stdout
    m = re.search(r"^\s*---\n(.*?)^\.\.\.", txt, re.S | re.M)
    assert m, "no AMDGPU metadata in librcbf_steps.co"
    return yaml.safe_load(m.group(1))["amdhsa.kernels"]


def test_aql_kernarg_layout_matches_code_object():
    """Every k_safe_step instantiation the AQL path can dispatch takes exactly
    the argument block csrc/rcbf_aql.hip writes (SafeStepArgs): 16 8-B
    scalars / pointers, auto_reset, seed, env_offset, the 240-B rcbf_params by
    value, prior_cols, the stamp pointer -- no hidden arguments -- and uses no
    scratch (checked again against the loaded symbols by rcbf_aql_open)."""
    from rcbf_amd import _lib
    want = [(8 * i, 8) for i in range(16)] + [(128, 4), (136, 8), (144, 8), (152, ctypes.sizeof(_lib.RcbfParams)),
                                              (392, 4), (400, 8)]
    ks = [k for k in _steps_code_object_kernels() if k[".name"].startswith("_ZN4rcbf11k_safe_step")]
    # solver x mode/hazards x workgroup size x (product, span)
    assert len(ks) >= 3 * 9 * 2
    for k in ks:
        assert k[".kernarg_segment_size"] == 408, k[".name"]
        assert [(a[".offset"], a[".size"]) for a in k[".args"]] == want, k[".name"]
        assert all(not a[".value_kind"].startswith("hidden") for a in k[".args"]), k[".name"]
        assert k[".private_segment_fixed_size"] == 0, k[".name"]


def test_aql_entry_points_reject_bad_arguments_without_gpu():
    from rcbf_amd import _lib
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.rcbf_aql_open(0, None, 0, None) == 1003
    assert lib.rcbf_aql_open(-1, None, 0, ctypes.byref(h)) == 1002  # no such HIP device (none here)
    assert lib.rcbf_aql_run(None, 0) == 1003
    assert lib.rcbf_aql_plan_free(None) == 0
    assert lib.rcbf_aql_close(None) == 0
