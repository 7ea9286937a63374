// rcbf_pyfast.cpp -- CPython binding of the per-step entry points of
// include/rcbf_hip.h for eager Python callers: rcbf_safe_step,
// rcbf_safe_step_seq, rcbf_env_step_sync and rcbf_gp_obs_safe_action.
//
// BatchedEnv.safe_step is called once per env step; through ctypes its 21
// arguments cost ~4 us of host time per call, comparable to the ~4.3 us
// kernel.  This module takes the same arguments as plain Python ints (device
// pointers, 0 for NULL) through METH_FASTCALL and calls the C-ABI directly.
//
// It does not link librcbf_hip.so: bind() receives the addresses of the
// entry points from the library ctypes loaded (rcbf_amd._lib, which honours
// RCBF_HIP_LIB), so both bindings always call into the same library copy.
// No torch types cross it.
#include <Python.h>

#include "rcbf_hip.h"

namespace {

using SafeStepFn = decltype(&rcbf_safe_step);
using SafeStepSeqFn = decltype(&rcbf_safe_step_seq);
using EnvStepSyncFn = decltype(&rcbf_env_step_sync);
using GpSafeActionFn = decltype(&rcbf_gp_obs_safe_action);

SafeStepFn g_safe_step = nullptr;
SafeStepSeqFn g_safe_step_seq = nullptr;
EnvStepSyncFn g_env_step_sync = nullptr;
GpSafeActionFn g_gp_safe_action = nullptr;

bool as_u64(PyObject* o, unsigned long long* v) {
    if (o == Py_None) {
        *v = 0;
        return true;
    }
    *v = PyLong_AsUnsignedLongLongMask(o);
    return !(*v == (unsigned long long)-1 && PyErr_Occurred());
}

bool args_u64(PyObject* const* args, Py_ssize_t nargs, Py_ssize_t want, unsigned long long* a, const char* name) {
    if (nargs != want) {
        PyErr_Format(PyExc_TypeError, "%s expects %zd arguments, got %zd", name, want, nargs);
        return false;
    }
    for (Py_ssize_t k = 0; k < want; ++k)
        if (!as_u64(args[k], &a[k])) return false;
    return true;
}

bool bound(const void* fn, const char* name) {
    if (fn) return true;
    PyErr_Format(PyExc_RuntimeError, "_rcbf_fast.%s: call bind() with the loaded library's entry points first", name);
    return false;
}

// bind(addr_safe_step, addr_safe_step_seq, addr_env_step_sync, addr_gp_obs_safe_action) -> None
PyObject* bind(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
    unsigned long long a[4];
    if (!args_u64(args, nargs, 4, a, "bind")) return nullptr;
    g_safe_step = reinterpret_cast<SafeStepFn>(a[0]);
    g_safe_step_seq = reinterpret_cast<SafeStepSeqFn>(a[1]);
    g_env_step_sync = reinterpret_cast<EnvStepSyncFn>(a[2]);
    g_gp_safe_action = reinterpret_cast<GpSafeActionFn>(a[3]);
    Py_RETURN_NONE;
}

// bound() -> the entry-point addresses bind() stored, in bind()'s order
PyObject* bound_addrs(PyObject*, PyObject* const*, Py_ssize_t nargs) {
    if (nargs != 0) {
        PyErr_SetString(PyExc_TypeError, "bound() takes no arguments");
        return nullptr;
    }
    return Py_BuildValue("(KKKK)", (unsigned long long)(uintptr_t)g_safe_step,
                         (unsigned long long)(uintptr_t)g_safe_step_seq,
                         (unsigned long long)(uintptr_t)g_env_step_sync,
                         (unsigned long long)(uintptr_t)g_gp_safe_action);
}

// gp_obs_safe_action(prm, model, obs, u_rl, workspace, stream, host_block, seq) -> int: rcbf_gp_obs_safe_action
// at B = 1 with the action, the QP status and the completion word in one pinned host block (bytes 0, 32, 64);
// returns once the word reads seq (the action is then on the host)
PyObject* gp_obs_safe_action(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
    unsigned long long a[8];
    if (!args_u64(args, nargs, 8, a, "gp_obs_safe_action") ||
        !bound((const void*)g_gp_safe_action, "gp_obs_safe_action"))
        return nullptr;
    int rc;
    char* host = reinterpret_cast<char*>(a[6]);
    Py_BEGIN_ALLOW_THREADS
    rc = g_gp_safe_action(reinterpret_cast<const rcbf_params*>(a[0]), reinterpret_cast<const rcbf_gp_model*>(a[1]), 1,
                          reinterpret_cast<const float*>(a[2]), reinterpret_cast<const float*>(a[3]), nullptr,
                          nullptr, nullptr, reinterpret_cast<float*>(host), reinterpret_cast<uint32_t*>(host + 64),
                          (uint32_t)a[7], reinterpret_cast<int32_t*>(host + 32), nullptr,
                          reinterpret_cast<float*>(a[4]), reinterpret_cast<hipStream_t>(a[5]));
    Py_END_ALLOW_THREADS
    return PyLong_FromLong(rc);
}

// safe_step(prm, B, x, aux, step, episode, u_rl, mu, sigma, obs, u_out, reward,
//           cost, done, goal_met, status, fail_flag, auto_reset, seed, env_offset,
//           stream) -> int   (rcbf_safe_step's return code)
PyObject* safe_step(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
    unsigned long long a[21];
    if (!args_u64(args, nargs, 21, a, "safe_step") || !bound((const void*)g_safe_step, "safe_step")) return nullptr;
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = g_safe_step(reinterpret_cast<const rcbf_params*>(a[0]), (int64_t)a[1], reinterpret_cast<double*>(a[2]),
                     reinterpret_cast<double*>(a[3]), reinterpret_cast<int32_t*>(a[4]),
                     reinterpret_cast<uint32_t*>(a[5]), reinterpret_cast<const float*>(a[6]),
                     reinterpret_cast<const float*>(a[7]), reinterpret_cast<const float*>(a[8]),
                     reinterpret_cast<float*>(a[9]), reinterpret_cast<float*>(a[10]), reinterpret_cast<float*>(a[11]),
                     reinterpret_cast<float*>(a[12]), reinterpret_cast<uint8_t*>(a[13]),
                     reinterpret_cast<uint8_t*>(a[14]), reinterpret_cast<int32_t*>(a[15]),
                     reinterpret_cast<int32_t*>(a[16]), (int32_t)a[17], (uint64_t)a[18], (int64_t)a[19],
                     reinterpret_cast<hipStream_t>(a[20]));
    Py_END_ALLOW_THREADS
    return PyLong_FromLong(rc);
}

// safe_step_seq(prm, B, K, x, aux, step, episode, u_rl_ptrs (sequence of
//               ints), mu, sigma, obs, u_out, reward, cost, done, goal_met,
//               status, fail_flag, auto_reset, seed, env_offset, stream) -> int
PyObject* safe_step_seq(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
    if (nargs != 22) {
        PyErr_Format(PyExc_TypeError, "safe_step_seq expects 22 arguments, got %zd", nargs);
        return nullptr;
    }
    if (!bound((const void*)g_safe_step_seq, "safe_step_seq")) return nullptr;
    unsigned long long a[22];
    for (int k = 0; k < 22; ++k)
        if (k != 7 && !as_u64(args[k], &a[k])) return nullptr;
    PyObject* seq = PySequence_Fast(args[7], "u_rl_ptrs must be a sequence of device pointers");
    if (!seq) return nullptr;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
    if (n < 1 || n > 4096) {
        Py_DECREF(seq);
        PyErr_SetString(PyExc_ValueError, "u_rl_ptrs must hold 1..4096 pointers");
        return nullptr;
    }
    const float* ptrs[4096];
    for (Py_ssize_t j = 0; j < n; ++j) {
        unsigned long long v;
        if (!as_u64(PySequence_Fast_GET_ITEM(seq, j), &v)) {
            Py_DECREF(seq);
            return nullptr;
        }
        ptrs[j] = reinterpret_cast<const float*>(v);
    }
    Py_DECREF(seq);
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = g_safe_step_seq(reinterpret_cast<const rcbf_params*>(a[0]), (int64_t)a[1], (int32_t)a[2],
                         reinterpret_cast<double*>(a[3]), reinterpret_cast<double*>(a[4]),
                         reinterpret_cast<int32_t*>(a[5]), reinterpret_cast<uint32_t*>(a[6]), ptrs, (int32_t)n,
                         reinterpret_cast<const float*>(a[8]), reinterpret_cast<const float*>(a[9]),
                         reinterpret_cast<float*>(a[10]), reinterpret_cast<float*>(a[11]),
                         reinterpret_cast<float*>(a[12]), reinterpret_cast<float*>(a[13]),
                         reinterpret_cast<uint8_t*>(a[14]), reinterpret_cast<uint8_t*>(a[15]),
                         reinterpret_cast<int32_t*>(a[16]), reinterpret_cast<int32_t*>(a[17]), (int32_t)a[18],
                         (uint64_t)a[19], (int64_t)a[20], reinterpret_cast<hipStream_t>(a[21]));
    Py_END_ALLOW_THREADS
    return PyLong_FromLong(rc);
}

// env_step_sync(prm, B, x, aux, step, episode, action_host, action_f64,
//               packed_host, auto_reset, seed, env_offset, stream) -> int
PyObject* env_step_sync(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
    unsigned long long a[13];
    if (!args_u64(args, nargs, 13, a, "env_step_sync") || !bound((const void*)g_env_step_sync, "env_step_sync"))
        return nullptr;
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = g_env_step_sync(reinterpret_cast<const rcbf_params*>(a[0]), (int64_t)a[1], reinterpret_cast<double*>(a[2]),
                         reinterpret_cast<double*>(a[3]), reinterpret_cast<int32_t*>(a[4]),
                         reinterpret_cast<uint32_t*>(a[5]), reinterpret_cast<const void*>(a[6]), (int32_t)a[7],
                         reinterpret_cast<double*>(a[8]), (int32_t)a[9], (uint64_t)a[10], (int64_t)a[11],
                         reinterpret_cast<hipStream_t>(a[12]));
    Py_END_ALLOW_THREADS
    return PyLong_FromLong(rc);
}

#define RCBF_FASTCALL(f) reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(f))
PyMethodDef kMethods[] = {
    {"bind", RCBF_FASTCALL(bind), METH_FASTCALL, "bind the entry points of the loaded librcbf_hip.so"},
    {"bound", RCBF_FASTCALL(bound_addrs), METH_FASTCALL, "the entry-point addresses bind() stored"},
    {"safe_step", RCBF_FASTCALL(safe_step), METH_FASTCALL, "rcbf_safe_step with integer pointer arguments"},
    {"safe_step_seq", RCBF_FASTCALL(safe_step_seq), METH_FASTCALL,
     "rcbf_safe_step_seq with integer pointer arguments and a sequence of u_rl pointers"},
    {"env_step_sync", RCBF_FASTCALL(env_step_sync), METH_FASTCALL,
     "rcbf_env_step_sync (launch + stream synchronise) with integer pointer arguments"},
    {"gp_obs_safe_action", RCBF_FASTCALL(gp_obs_safe_action), METH_FASTCALL,
     "rcbf_gp_obs_safe_action at B = 1 into a pinned host block, with integer pointer arguments"},
    {nullptr, nullptr, 0, nullptr}};
#undef RCBF_FASTCALL

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_rcbf_fast", "CPython binding of the per-step C-ABI entry points", -1,
                       kMethods, nullptr, nullptr, nullptr, nullptr};

}  // namespace

extern "C" PyMODINIT_FUNC PyInit__rcbf_fast(void) { return PyModule_Create(&kModule); }
