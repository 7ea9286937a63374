// rcbf_aql.hip -- the fused safe step dispatched as raw AQL packets on a
// user-mode HSA queue owned by the library (host code only; no kernels here).
//
// Why: a step of the hot path is ~3.6 us of GPU time, and the HIP launch path
// costs more than that around a short sequence of them: hipGraphLaunch spends
// ~16-25 us of host time on a 20-node graph and the first kernel starts ~17 us
// after the event recorded before it (profiles/README.md, r02 narrative);
// hipLaunchKernel costs ~5 us of host time per launch.  The driver's 20-step
// bench line therefore spends ~30 % of its wall time outside the kernels.
//
// What: the kernels are the SAME machine code HIP launches -- the gfx950 code
// object embedded in rcbf_env.o, unbundled at build time into
// librcbf_steps.co next to librcbf_hip.so -- loaded once into an HSA
// executable.  A "plan" is the AQL analogue of an instantiated hipGraph: the
// kernel-argument blocks of K steps written once into device memory and the K
// dispatch packets pre-built on the host.  Running a plan copies the K packets
// into the queue's ring (60 B each + an atomic header store), rings the
// doorbell once and waits on the last packet's completion signal, so the
// host-side cost of K dispatches is ~1 us and the packet processor starts the
// first kernel as soon as it reads the packet.  Every packet has the barrier
// bit: step j + 1 starts after step j has completed, exactly like K launches
// on one in-order stream.  Memory scopes: the last packet releases at system
// scope (the host reads the completion signal; HIP work after the call sees
// the results), the packets between
// acquire and release at agent scope, which on gfx950 writes the XCD L2s back
// and invalidates them between steps as HIP's in-order stream does.  The first
// packet acquires at agent scope: every input of the step is device memory
// written by device work or copies that completed before the run (a system-
// scope acquire there cost the first step ~3 us: profiles/r06/aql_fences_r06e.json).
//
// Reference interface this serves: env.step() of the batched env inside the
// SAC loop (main.py:93-95, sac_cbf.py:218-238) -- a synchronous call, like a
// gym step: rcbf_aql_run returns when the K steps have completed.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <dlfcn.h>
#include <immintrin.h>
#include <time.h>

#include <atomic>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "rcbf_common.hpp"
#include "rcbf_hip.h"

namespace {

using namespace rcbf;

// Kernel-argument block of rcbf::k_safe_step (rcbf_safe_step.hpp), in the
// order and at the offsets of its parameter list (the AMDGPU kernarg ABI:
// every argument at its natural alignment, by-value structs included).  The
// kernel reads no hidden arguments (its code-object metadata lists none and
// its kernarg_segment_size is 408), which rcbf_aql_open checks against the
// loaded code object before any dispatch; tests/test_abi_cpu.py checks the
// offsets against the metadata of librcbf_steps.co on the CPU.
struct SafeStepArgs {
    int64_t B;
    double* x;
    double* aux;
    int32_t* step;
    const float* u_rl;
    uint32_t* episode;
    const float* mu;
    const float* sigma;
    float* obs_out;
    float* u_out;
    float* reward;
    float* cost;
    uint8_t* done;
    uint8_t* goal_met;
    int32_t* status_out;
    int32_t* fail_flag;
    int32_t auto_reset;
    uint64_t seed;
    int64_t off;
    rcbf_params prm;
    int32_t prior_cols;
    unsigned long long* stamp_buf;
};
static_assert(offsetof(SafeStepArgs, auto_reset) == 128, "kernarg layout");
static_assert(offsetof(SafeStepArgs, seed) == 136, "kernarg layout");
static_assert(offsetof(SafeStepArgs, prm) == 152, "kernarg layout");
static_assert(offsetof(SafeStepArgs, prior_cols) == 392, "kernarg layout");
static_assert(offsetof(SafeStepArgs, stamp_buf) == 400, "kernarg layout");
static_assert(sizeof(SafeStepArgs) == RCBF_AQL_SAFE_STEP_KERNARG_BYTES, "kernarg layout");

struct KernelInfo {
    std::string name;  // mangled symbol without ".kd"
    uint64_t object = 0;
    uint32_t kernarg_bytes = 0, group_bytes = 0, private_bytes = 0;
};

constexpr uint32_t kQueueSize = 4096;  // packets (power of two); a plan longer than this is fed in chunks
constexpr size_t kArgStride = 512;     // bytes per step's kernarg block (>= 408, 64-B multiple)

uint64_t now_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

}  // namespace

struct rcbf_aql {
    int device = -1;
    hsa_agent_t agent{};
    hsa_queue_t* queue = nullptr;
    hsa_code_object_reader_t reader{};
    hsa_executable_t exe{};
    bool have_reader = false, have_exe = false, hsa_up = false;
    std::vector<char> code;
    std::vector<KernelInfo> kernels;
    std::atomic<int> queue_error{0};
    int profiling = 0;
};

struct rcbf_aql_plan {
    rcbf_aql* q = nullptr;
    int device = -1;  // the queue's HIP device (rcbf_aql_plan_free does not read q: a plan may outlive it)
    int32_t K = 0;
    void* kernargs = nullptr;                       // K * kArgStride bytes of device memory
    std::vector<hsa_kernel_dispatch_packet_t> pkt;  // pre-built packets (header written last, atomically)
    std::vector<hsa_signal_t> sig;                  // completion signals: one per packet (profiled) or one
    int profiled = 0;
};

namespace {

void queue_error_cb(hsa_status_t status, hsa_queue_t*, void* data) {
    auto* q = static_cast<rcbf_aql*>(data);
    q->queue_error.store((int)status);
}

struct AgentSearch {
    uint32_t bdf;
    uint32_t domain;
    hsa_agent_t found{};
    bool ok = false;
};

hsa_status_t find_agent(hsa_agent_t a, void* data) {
    auto* s = static_cast<AgentSearch*>(data);
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
        return HSA_STATUS_SUCCESS;
    uint32_t bdf = 0, dom = 0;
    if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) != HSA_STATUS_SUCCESS)
        return HSA_STATUS_SUCCESS;
    hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
    // BDFID = bus << 8 | device << 3 | function
    if ((bdf >> 3) == (s->bdf >> 3) && dom == s->domain) {
        s->found = a;
        s->ok = true;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

hsa_status_t collect_kernel(hsa_executable_t, hsa_agent_t, hsa_executable_symbol_t sym, void* data) {
    auto* q = static_cast<rcbf_aql*>(data);
    hsa_symbol_kind_t kind;
    if (hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &kind) != HSA_STATUS_SUCCESS ||
        kind != HSA_SYMBOL_KIND_KERNEL)
        return HSA_STATUS_SUCCESS;
    uint32_t len = 0;
    hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &len);
    std::string name(len, '\0');
    hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_NAME, name.data());
    if (name.size() > 3 && name.compare(name.size() - 3, 3, ".kd") == 0) name.resize(name.size() - 3);
    KernelInfo k;
    k.name = name;
    hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.object);
    hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k.kernarg_bytes);
    hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.group_bytes);
    hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.private_bytes);
    q->kernels.push_back(std::move(k));
    return HSA_STATUS_SUCCESS;
}

// Itanium mangling of rcbf::k_safe_step<SOLVER, MODE, K, false, BS, SPAN>'s
// name and template arguments; the parameter list that follows is the one
// SafeStepArgs mirrors (checked by size at open and by the CPU test).
std::string safe_step_prefix(int solver, int mode, int k, int bs, bool span) {
    char buf[128];
    snprintf(buf, sizeof buf, "_ZN4rcbf11k_safe_stepILi%dELi%dELi%dELb0ELi%dELb%dEEEv", solver, mode, k, bs,
             span ? 1 : 0);
    return buf;
}

const KernelInfo* find_kernel(const rcbf_aql* q, const std::string& prefix) {
    const KernelInfo* hit = nullptr;
    for (const auto& k : q->kernels)
        if (k.name.compare(0, prefix.size(), prefix) == 0) {
            if (hit) return nullptr;  // ambiguous
            hit = &k;
        }
    return hit;
}

int hsa_rc(hsa_status_t s) { return s == HSA_STATUS_SUCCESS ? 0 : RCBF_E_HSA; }

// Current HIP device set to `dev` for the scope (kernarg copies, CU count).
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

void destroy(rcbf_aql* q) {
    if (!q) return;
    if (q->queue) hsa_queue_destroy(q->queue);
    if (q->have_exe) hsa_executable_destroy(q->exe);
    if (q->have_reader) hsa_code_object_reader_destroy(q->reader);
    if (q->hsa_up) hsa_shut_down();
    delete q;
}

}  // namespace

extern "C" {

int rcbf_aql_open(int32_t device, const char* code_object_path, int32_t flags, rcbf_aql** out) {
    if (!out) return RCBF_E_NULL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return RCBF_E_BAD_SHAPE;
    std::string path;
    if (code_object_path && *code_object_path) {
        path = code_object_path;
    } else {  // librcbf_steps.co next to this library
        Dl_info info;
        if (!dladdr((void*)&rcbf_aql_open, &info) || !info.dli_fname) return RCBF_E_NULL;
        path = info.dli_fname;
        const size_t slash = path.rfind('/');
        path = (slash == std::string::npos ? std::string(".") : path.substr(0, slash)) + "/librcbf_steps.co";
    }
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return RCBF_E_NULL;
    auto* q = new rcbf_aql();
    q->device = device;
    q->profiling = (flags & RCBF_AQL_PROFILE) ? 1 : 0;
    fseek(f, 0, SEEK_END);
    const long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    q->code.resize(n > 0 ? (size_t)n : 0);
    const bool read_ok = n > 0 && fread(q->code.data(), 1, (size_t)n, f) == (size_t)n;
    fclose(f);
    if (!read_ok) {
        delete q;
        return RCBF_E_BAD_SHAPE;
    }
    int rc = hsa_rc(hsa_init());
    if (rc) {
        delete q;
        return rc;
    }
    q->hsa_up = true;
    // the HSA agent of HIP device `device`, matched by PCI location (HIP's device
    // ordinals follow HIP_VISIBLE_DEVICES, HSA's agent list does not)
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
        destroy(q);
        return RCBF_E_HSA;
    }
    AgentSearch s{(uint32_t)((prop.pciBusID << 8) | (prop.pciDeviceID << 3)), (uint32_t)prop.pciDomainID};
    hsa_iterate_agents(find_agent, &s);
    if (!s.ok) {
        destroy(q);
        return RCBF_E_HSA;
    }
    q->agent = s.found;
    rc = hsa_rc(hsa_code_object_reader_create_from_memory(q->code.data(), q->code.size(), &q->reader));
    if (!rc) q->have_reader = true;
    if (!rc)
        rc = hsa_rc(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr,
                                              &q->exe));
    if (!rc) q->have_exe = true;
    if (!rc) rc = hsa_rc(hsa_executable_load_agent_code_object(q->exe, q->agent, q->reader, nullptr, nullptr));
    if (!rc) rc = hsa_rc(hsa_executable_freeze(q->exe, nullptr));
    if (!rc) rc = hsa_rc(hsa_executable_iterate_agent_symbols(q->exe, q->agent, collect_kernel, q));
    // every k_safe_step instantiation in the code object must take exactly the
    // argument block SafeStepArgs describes
    int n_steps = 0;
    for (const auto& k : q->kernels)
        if (k.name.compare(0, 21, "_ZN4rcbf11k_safe_step") == 0) {
            ++n_steps;
            if (k.kernarg_bytes != sizeof(SafeStepArgs) || k.private_bytes != 0) rc = RCBF_E_BAD_SHAPE;
        }
    if (!rc && n_steps == 0) rc = RCBF_E_BAD_MODE;
    if (!rc)
        rc = hsa_rc(hsa_queue_create(q->agent, kQueueSize, HSA_QUEUE_TYPE_SINGLE, queue_error_cb, q, UINT32_MAX,
                                     UINT32_MAX, &q->queue));
    if (!rc && q->profiling) rc = hsa_rc(hsa_amd_profiling_set_profiler_enabled(q->queue, 1));
    if (rc) {
        destroy(q);
        return rc;
    }
    *out = q;
    return 0;
}

int rcbf_aql_close(rcbf_aql* q) {
    destroy(q);
    return 0;
}

int rcbf_aql_kernel_count(const rcbf_aql* q) { return q ? (int)q->kernels.size() : RCBF_E_NULL; }

int rcbf_aql_safe_step_plan(rcbf_aql* q, const rcbf_params* prm, int64_t B, int32_t K, double* x, double* aux,
                            int32_t* step, uint32_t* episode, const float* const* u_rl_seq, int32_t n_u_rl,
                            const float* mu, const float* sigma, int32_t prior_cols, float* obs_out, float* u_out,
                            float* reward, float* cost, uint8_t* done, uint8_t* goal_met, int32_t* status_out,
                            int32_t* fail_flag, int32_t auto_reset, uint64_t seed, int64_t env_offset,
                            uint64_t* span_out, int32_t flags, rcbf_aql_plan** out) {
    if (!q || !out) return RCBF_E_NULL;
    *out = nullptr;
    if (int e = check_prm(prm)) return e;
    if (B <= 0 || K <= 0 || n_u_rl <= 0 || B > INT32_MAX) return RCBF_E_BAD_SHAPE;
    if (!u_rl_seq) return RCBF_E_NULL;
    for (int32_t j = 0; j < n_u_rl; ++j)
        if (!u_rl_seq[j]) return RCBF_E_NULL;
    if (!x || !aux || !step || !obs_out || !u_out || !reward || !cost || !done) return RCBF_E_NULL;
    if ((((uintptr_t)obs_out) & 7) || (((uintptr_t)x) & 15)) return RCBF_E_BAD_SHAPE;
    if (prior_cols && prm->mode == RCBF_MODE_SIMULATED_CARS && mu) return RCBF_E_BAD_SHAPE;
    if (span_out && (((uintptr_t)span_out) & 15)) return RCBF_E_BAD_SHAPE;
    if (span_out && prm->solver != RCBF_SOLVER_ACTIVE_SET) return RCBF_E_BAD_MODE;
    // RCBF_AQL_PROFILE: a completion signal (timestamps) on every packet; RCBF_AQL_PROFILE_ENDS: on the first
    // and the last only, so the run is timed end to end without a signal between steps (each one adds
    // ~1.5 us to its step: profiles/r06/aql_dispatch_signal_cost)
    const bool ends = (flags & RCBF_AQL_PROFILE_ENDS) != 0;
    const bool profiled = (flags & RCBF_AQL_PROFILE) != 0 || ends;
    if (profiled && !q->profiling) return RCBF_E_BAD_MODE;
    DeviceGuard guard(q->device);
    // the launch rcbf_safe_step would make: solver, mode, hazards, workgroup size
    const int solver = prm->solver;
    const int mode = prm->mode;
    const int k = mode == RCBF_MODE_SIMULATED_CARS ? 1 : prm->num_hazards;
    const int bs = solver == RCBF_SOLVER_ACTIVE_SET ? block_for_envs(B) : 256;
    const KernelInfo* ki = find_kernel(q, safe_step_prefix(solver, mode, k, bs, span_out != nullptr));
    if (!ki || ki->kernarg_bytes != sizeof(SafeStepArgs)) return RCBF_E_BAD_MODE;
    const uint64_t groups = (uint64_t)grid_for_envs(B, bs);

    auto* p = new rcbf_aql_plan();
    p->q = q;
    p->device = q->device;
    p->K = K;
    p->profiled = ends ? 2 : profiled ? 1 : 0;
    std::vector<unsigned char> host((size_t)K * kArgStride, 0);
    for (int32_t j = 0; j < K; ++j) {
        SafeStepArgs a;
        std::memset(&a, 0, sizeof a);
        a.B = B;
        a.x = x;
        a.aux = aux;
        a.step = step;
        a.u_rl = u_rl_seq[j % n_u_rl];
        a.episode = episode;
        a.mu = mu;
        a.sigma = sigma;
        a.obs_out = obs_out;
        a.u_out = u_out;
        a.reward = reward;
        a.cost = cost;
        a.done = done;
        a.goal_met = goal_met;
        a.status_out = status_out;
        a.fail_flag = fail_flag;
        a.auto_reset = auto_reset;
        a.seed = seed;
        a.off = env_offset;
        a.prm = *prm;
        a.prior_cols = prior_cols ? 1 : 0;
        // step j's stamps: its own block of 4 ceil(B / 64) words
        a.stamp_buf = span_out ? reinterpret_cast<unsigned long long*>(span_out) + (size_t)j * 4 * ((B + 63) / 64)
                               : nullptr;
        std::memcpy(host.data() + (size_t)j * kArgStride, &a, sizeof a);
    }
    int rc = (int)hipMalloc(&p->kernargs, host.size());
    if (!rc) rc = (int)hipMemcpy(p->kernargs, host.data(), host.size(), hipMemcpyHostToDevice);
    const int nsig = p->profiled == 1 ? K : p->profiled == 2 ? 2 : 1;
    for (int j = 0; !rc && j < nsig; ++j) {
        hsa_signal_t s;
        rc = hsa_rc(hsa_signal_create(1, 0, nullptr, &s));
        if (!rc) p->sig.push_back(s);
    }
    if (rc) {
        rcbf_aql_plan_free(p);
        return rc;
    }
    p->pkt.resize(K);
    for (int32_t j = 0; j < K; ++j) {
        hsa_kernel_dispatch_packet_t& d = p->pkt[j];
        std::memset(&d, 0, sizeof d);
        int acq = j == 0 && (flags & RCBF_AQL_FIRST_ACQUIRE_SYSTEM) ? HSA_FENCE_SCOPE_SYSTEM : HSA_FENCE_SCOPE_AGENT;
        int rel = j == K - 1 && !(flags & RCBF_AQL_LAST_RELEASE_AGENT) ? HSA_FENCE_SCOPE_SYSTEM : HSA_FENCE_SCOPE_AGENT;
        if ((flags & (RCBF_AQL_STUDY_MID_NOFENCE | RCBF_AQL_STUDY_MID_NOACQ)) && j > 0) acq = HSA_FENCE_SCOPE_NONE;
        if ((flags & (RCBF_AQL_STUDY_MID_NOFENCE | RCBF_AQL_STUDY_MID_NOREL)) && j < K - 1) rel = HSA_FENCE_SCOPE_NONE;
        d.header = (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                              (1 << HSA_PACKET_HEADER_BARRIER) | (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                              (rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
        d.setup = (uint16_t)(1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS);
        d.workgroup_size_x = (uint16_t)bs;
        d.workgroup_size_y = 1;
        d.workgroup_size_z = 1;
        d.grid_size_x = (uint32_t)(groups * (uint64_t)bs);
        d.grid_size_y = 1;
        d.grid_size_z = 1;
        d.private_segment_size = ki->private_bytes;
        d.group_segment_size = ki->group_bytes;
        d.kernel_object = ki->object;
        d.kernarg_address = static_cast<unsigned char*>(p->kernargs) + (size_t)j * kArgStride;
        if (p->profiled == 1)
            d.completion_signal = p->sig[j];
        else if (p->profiled == 2 && (j == 0 || j == K - 1))
            d.completion_signal = p->sig[j == 0 ? 0 : 1];
        else if (j == K - 1)
            d.completion_signal = p->sig[0];
        else
            d.completion_signal.handle = 0;
    }
    *out = p;
    return 0;
}

}  // extern "C"

namespace {

// Copy packets j, j + 1, ... of plan p into its queue's ring, as many as the ring has room for right now,
// and ring the doorbell once for them; returns the new j (unchanged when the ring is full).
int32_t feed(rcbf_aql_plan* p, int32_t j) {
    hsa_queue_t* queue = p->q->queue;
    const uint64_t mask = queue->size - 1;
    auto* ring = static_cast<hsa_kernel_dispatch_packet_t*>(queue->base_address);
    const uint64_t rd = hsa_queue_load_read_index_scacquire(queue);
    const uint64_t wr = hsa_queue_load_write_index_relaxed(queue);
    const uint64_t room = queue->size - (wr - rd);
    if (room == 0) return j;
    const int32_t n = (int32_t)std::min<uint64_t>(room, (uint64_t)(p->K - j));
    const uint64_t w = hsa_queue_add_write_index_relaxed(queue, (uint64_t)n);
    for (int32_t i = 0; i < n; ++i) {
        hsa_kernel_dispatch_packet_t* slot = &ring[(w + i) & mask];
        const hsa_kernel_dispatch_packet_t& src = p->pkt[j + i];
        std::memcpy(reinterpret_cast<char*>(slot) + 4, reinterpret_cast<const char*>(&src) + 4, sizeof(src) - 4);
        __atomic_store_n(reinterpret_cast<uint32_t*>(slot), (uint32_t)src.header | ((uint32_t)src.setup << 16),
                         __ATOMIC_RELEASE);
    }
    hsa_signal_store_screlease(queue->doorbell_signal, (hsa_signal_value_t)(w + n - 1));
    return j + n;
}

// Busy-wait for plan p's last completion signal (a synchronous step: the host has nothing else to do, and
// a sleeping wait adds its wake-up latency to every call).
int wait_done(rcbf_aql_plan* p, uint64_t t_end) {
    const hsa_signal_t last = p->sig.back();
    for (;;) {
        const hsa_signal_value_t v =
            hsa_signal_wait_scacquire(last, HSA_SIGNAL_CONDITION_LT, 1, 1000000, HSA_WAIT_STATE_ACTIVE);
        if (v < 1) return p->q->queue_error.load() ? RCBF_E_HSA : 0;
        if (p->q->queue_error.load()) return RCBF_E_HSA;
        if (now_ns() > t_end) return RCBF_E_TIMEOUT;
    }
}

}  // namespace

extern "C" {

int rcbf_aql_run(rcbf_aql_plan* p, uint64_t timeout_us) {
    if (!p || !p->q || !p->q->queue) return RCBF_E_NULL;
    if (p->q->queue_error.load()) return RCBF_E_HSA;
    for (auto& s : p->sig) hsa_signal_store_relaxed(s, 1);
    const uint64_t t_end = now_ns() + (timeout_us ? timeout_us : 10000000ull) * 1000ull;
    // as many packets as the ring has room for (all of them unless K > the ring), then the rest as the
    // packet processor frees slots
    for (int32_t j = 0; j < p->K;) {
        const int32_t nj = feed(p, j);
        if (nj == j) {
            if (p->q->queue_error.load()) return RCBF_E_HSA;
            if (now_ns() > t_end) return RCBF_E_TIMEOUT;
            _mm_pause();
        }
        j = nj;
    }
    return wait_done(p, t_end);
}

int rcbf_aql_plan_times(const rcbf_aql_plan* p, uint64_t* start_end_ns) {
    if (!p || !start_end_ns) return RCBF_E_NULL;
    if (!p->profiled) return RCBF_E_BAD_MODE;
    uint64_t freq = 0;
    hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &freq);
    if (!freq) return RCBF_E_HSA;
    for (int32_t j = 0; j < p->K; ++j) {
        hsa_amd_profiling_dispatch_time_t t;
        int si = j;
        if (p->profiled == 2) {  // only the first and the last packets carry a signal
            start_end_ns[2 * j] = start_end_ns[2 * j + 1] = 0;
            if (j != 0 && j != p->K - 1) continue;
            si = j == 0 ? 0 : 1;
        }
        if (hsa_amd_profiling_get_dispatch_time(p->q->agent, p->sig[si], &t) != HSA_STATUS_SUCCESS) return RCBF_E_HSA;
        start_end_ns[2 * j] = (uint64_t)((long double)t.start * 1e9L / (long double)freq);
        start_end_ns[2 * j + 1] = (uint64_t)((long double)t.end * 1e9L / (long double)freq);
    }
    return 0;
}

int rcbf_aql_plan_free(rcbf_aql_plan* p) {
    if (!p) return 0;
    if (p->kernargs) {
        DeviceGuard guard(p->device);
        (void)hipFree(p->kernargs);
    }
    for (auto& s : p->sig) hsa_signal_destroy(s);
    delete p;
    return 0;
}

}  // extern "C"
