// rcbf_uni_pair.hip -- STUDY BUILD ONLY (not part of librcbf_hip.so): the
// unicycle fused safe step with TWO lanes per env, for
// scripts/uni_pair_study.py.  Built on demand into build/study/librcbf_uni_pair.so.
//
// Lanes 2e and 2e + 1 of a wave own env e (32 envs per wave, 2 waves per SIMD
// at B = 65 536).  The hazard rows and their live-row test -- the work of the
// step that is the same instructions on different data -- are split: lane h
// builds hazards j = 2 jj + h (uni_rows_diff_cs's arithmetic, so the rows are
// the product's bit for bit) and tests them; the halves are exchanged with
// one DPP row swap per value (quad_perm [1,0,3,2], no LDS) and both lanes
// solve the same rows in the same order (uni_qp_2d_masked: the product's
// solve from the exchanged live mask), so u is the product's bit for bit.
// Everything else (loads, the pre-step sincos and state32, the QP, the env
// step, the reset) runs in both lanes; lane 0 stores the state, lane 1 the
// per-env scalars, and the wave's 32 observation rows leave as 16-B chunks.
// SIMT lanes execute one instruction stream, so only data-parallel work can
// be split; the QP's candidates, the env step and the observation are one
// chain per env.
#include <hip/hip_runtime.h>

#include "../rcbf_safe_step.hpp"

using namespace rcbf;

namespace {

// the partner lane's value (lane ^ 1), one DPP move
__device__ __forceinline__ int pair_swap_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);  // quad_perm [1, 0, 3, 2]
}
__device__ __forceinline__ float pair_swap(float v) { return __int_as_float(pair_swap_i(__float_as_int(v))); }
__device__ __forceinline__ double pair_swap(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = pair_swap_i((int)(b & 0xFFFFFFFFLL)), hi = pair_swap_i((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// uni_qp_2d_core's live-row test of one row (max over the box of e_j > 0)
__device__ __forceinline__ unsigned uni_row_live_pair(float a0, float a1, float b, double L0, double U0, double L1,
                                                      double U1) {
    const double x0 = (double)a0, x1 = (double)a1;
    const double emax = (double)b + fmax(x0 * L0, x0 * U0) + fmax(x1 * L1, x1 * U1);
    return emax <= 0.0 ? 0u : 1u;
}

// this lane's hazard rows j = 2 jj + h (jj < KH), in the raw-solve form of
// uni_qp_2d_raw (a0 = G_j0, a1 = G_j1, b = -h_j), with uni_rows_diff_cs's
// operation order; chk as uni_qp_2d_raw's finiteness sum over these rows
template <int K, int KH>
__device__ __forceinline__ void pair_rows(const rcbf_params& prm, const float* xs, float c, float s, const float* u,
                                          const float* mu, const float* sig, int h, float* a0, float* a1, float* b,
                                          double& chk) {
#pragma clang fp contract(off)
    const float lp = (float)prm.l_p, g = (float)prm.gamma_b;
    float px = xs[0] + lp * c, py = xs[1] + lp * s;
    float g00 = c, g01 = -s * lp, g10 = s, g11 = c * lp;
    float mupx = g01 * mu[2] + mu[0], mupy = g11 * mu[2] + mu[1];
    float sgpx = fabsf(g01) * sig[2] + sig[0], sgpy = fabsf(g11) * sig[2] + sig[1];
    const float r2 = (float)((1.2 * prm.hazards_radius) * (1.2 * prm.hazards_radius));
    chk = 0.0;
#pragma unroll
    for (int jj = 0; jj < KH; ++jj) {
        const int je = 2 * jj, jo = 2 * jj + 1 < K ? 2 * jj + 1 : 2 * jj;  // a missing odd row repeats the even one
        const float ox = h ? (float)prm.hazards_xy[2 * jo] : (float)prm.hazards_xy[2 * je];
        const float oy = h ? (float)prm.hazards_xy[2 * jo + 1] : (float)prm.hazards_xy[2 * je + 1];
        float dx = px - ox, dy = py - oy;
        float hs = 0.5f * ((dx * dx + dy * dy) - r2);
        float A0 = dx * g00 + dy * g10;
        float A1 = dx * g01 + dy * g11;
        float t1 = dx * mupx + dy * mupy;
        float t2 = fabsf(dx) * sgpx + fabsf(dy) * sgpy;
        float t3 = A0 * u[0] + A1 * u[1];
        const float hj = g * ((hs * hs) * hs) + ((t1 - t2) + t3);
        a0[jj] = -A0;
        a1[jj] = -A1;
        b[jj] = -hj;
        chk += ((double)a0[jj] + (double)a1[jj]) + ((double)b[jj] + (double)(-1.0f));
    }
}

template <int K, int BS>
__global__ void __launch_bounds__(BS) k_uni_pair_step(int64_t B, double* __restrict__ x, double* __restrict__ aux,
                                                      int32_t* __restrict__ step, const float* __restrict__ u_rl,
                                                      uint32_t* __restrict__ episode, float* __restrict__ obs_out,
                                                      float* __restrict__ u_out, float* __restrict__ reward,
                                                      float* __restrict__ cost, uint8_t* __restrict__ done,
                                                      uint8_t* __restrict__ goal_met, int32_t* fail_flag,
                                                      int auto_reset, uint64_t seed, int64_t off, rcbf_params prm) {
    constexpr int MODE = RCBF_MODE_UNICYCLE;
    constexpr int KH = (K + 1) / 2;
    const int64_t tid = (int64_t)blockIdx.x * BS + threadIdx.x;
    const int h = threadIdx.x & 1;
    const int64_t i = tid >> 1;  // the pair shares i, so this exit is pair-uniform
    if (i >= B) return;
    double xs[3];
    load_state<MODE>(x, B, i, xs);
    double a = ld_in(&aux[i]);
    int st = ld_in(&step[i]);
    float us[2] = {ld_in(&u_rl[2 * i]), ld_in(&u_rl[2 * i + 1])};
    const bool ep_pre = episode && reset_foreseeable<MODE>(st, a);
    uint32_t ep0 = 0;
    if (ep_pre) ep0 = episode[i];
    float m[3], s[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        m[k] = 0.0f;
        s[k] = prior_sigma<MODE>(k);
    }
    // the pre-step sincos and state32 (both lanes)
    double c_th, s_th;
    sincos(xs[2], &s_th, &c_th);
    float s32[3], c_row, s_row;
    uni_state32_from_cs(xs, c_th, s_th, s32, c_row, s_row);
    // this lane's half of the hazard rows and their live bits
    float ra0[KH], ra1[KH], rb[KH];
    double chk;
    pair_rows<K, KH>(prm, s32, c_row, s_row, us, m, s, h, ra0, ra1, rb, chk);
    const float hK0 = (float)prm.u_max[0] - us[0], hK1 = -(float)prm.u_min[0] + us[0];
    const float hK2 = (float)prm.u_max[1] - us[1], hK3 = -(float)prm.u_min[1] + us[1];
    const double U0 = (double)hK0, L0 = -(double)hK1, U1 = (double)hK2, L1 = -(double)hK3;
    unsigned own = 0;
#pragma unroll
    for (int jj = 0; jj < KH; ++jj)
        if (2 * jj + h < K) own |= uni_row_live_pair(ra0[jj], ra1[jj], rb[jj], L0, U0, L1, U1) << (2 * jj + h);
    const unsigned mask = own | (unsigned)pair_swap_i((int)own);
    // both halves, in row order (row j from lane j & 1, slot j >> 1)
    float A0[K], A1[K], Bv[K];
#pragma unroll
    for (int jj = 0; jj < KH; ++jj) {
        const float p0 = pair_swap(ra0[jj]), p1 = pair_swap(ra1[jj]), pb = pair_swap(rb[jj]);
        A0[2 * jj] = h ? p0 : ra0[jj];
        A1[2 * jj] = h ? p1 : ra1[jj];
        Bv[2 * jj] = h ? pb : rb[jj];
        if (2 * jj + 1 < K) {
            A0[2 * jj + 1] = h ? ra0[jj] : p0;
            A1[2 * jj + 1] = h ? ra1[jj] : p1;
            Bv[2 * jj + 1] = h ? rb[jj] : pb;
        }
    }
    const double chk_all = chk + pair_swap(chk);
    double pd[3];
    diff_P<MODE>(pd);
    PMat<3, true> pm;
    pmat_set_diag<3>(pm, pd);
    double z[3];
    int status;
#if defined(RCBF_PAIR_CORE) && RCBF_PAIR_CORE  // study variant: the product's core (the mask recomputed from all rows)
    (void)mask;
    uni_qp_2d_core<K, float>(pm.P[0][0], pm.P[1][1], pm.P[2][2], pm.Pinv[0][0], pm.Pinv[1][1], A0, A1, Bv, L0, U0,
                             L1, U1, isfinite(chk_all), z, status);
#else
    uni_qp_2d_masked<K, float>(pm.P[0][0], pm.P[1][1], pm.P[2][2], pm.Pinv[0][0], pm.Pinv[1][1], A0, A1, Bv, mask,
                               L0, U0, L1, U1, isfinite(chk_all), z, status);
#endif
    float uf[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        float v = us[c] + (float)z[c];
        float lo = (float)prm.u_min[c], hi = (float)prm.u_max[c];
        uf[c] = fminf(fmaxf(v, lo), hi);  // torch.clamp (diff_cbf_qp.py:77)
    }
    // the env step, the reset (both lanes)
    UniStepOut o;
    uni_env_step_cs<float, K>(prm, xs, a, st, uf, c_th, s_th, o);
    const float rew = (float)o.reward, cst = (float)o.cost;
    const bool dn = o.done, gm = o.goal;
    double oc[4] = {o.c, o.s, o.gd, 1.0};
    if (auto_reset && dn) {
        const uint32_t ep = episode ? (ep_pre ? ep0 : episode[i]) + 1u : 0u;
        if (episode && h == 0) episode[i] = ep;
        env_reset_one<MODE>(nullptr, i, seed, off, ep, xs, a, st);
        oc[0] = 1.0;
        oc[1] = 0.0;
        oc[2] = a;
    }
    if (h == 0) {
        store_state<MODE>(x, B, i, xs);
        st_out(&aux[i], a);
        st_out(&step[i], st);
        report(status, nullptr, i, fail_flag);
    } else {
        st_out2(&u_out[2 * i], uf[0], uf[1]);
        st_out(&reward[i], rew);
        st_out(&cost[i], cst);
        st_out(&done[i], (uint8_t)dn);
        if (goal_met) st_out(&goal_met[i], (uint8_t)gm);
    }
    // the wave's 32 observation rows (896 B) through LDS, out as 56 chunks of 16 B
    __shared__ float obs_stage[BS / 64][32 * 7];
    float* lds = obs_stage[threadIdx.x >> 6];
    const int lane = threadIdx.x & 63;
    const int64_t i0 = i - (lane >> 1);
    const bool full = (i0 + 32 <= B) && ((reinterpret_cast<uintptr_t>(obs_out) & 15) == 0);
    if (!full) {
        if (h == 0) store_obs32<MODE>(obs_out, i, xs, oc);
        return;
    }
    if (h == 0) {
        double ob[7];
        uni_obs_cs(xs, oc[0], oc[1], oc[2], ob);
#pragma unroll
        for (int k = 0; k < 7; ++k) lds[(lane >> 1) * 7 + k] = (float)ob[k];
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < 56) {
        const float4 v = reinterpret_cast<const float4*>(lds)[lane];
        st_out4<false>(obs_out + i0 * 7 + 4 * lane, v);
    }
}

}  // namespace

extern "C" int rcbf_study_uni_pair_step(const rcbf_params* prm, int64_t B, double* x, double* aux, int32_t* step,
                                        uint32_t* episode, const float* u_rl, float* obs_out, float* u_out,
                                        float* reward, float* cost, uint8_t* done, uint8_t* goal_met,
                                        int32_t* fail_flag, int32_t auto_reset, uint64_t seed, int64_t off,
                                        int32_t bs, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (prm->mode != RCBF_MODE_UNICYCLE || prm->solver != RCBF_SOLVER_ACTIVE_SET) return RCBF_E_BAD_MODE;
    if (B <= 0) return RCBF_E_BAD_SHAPE;
    if (bs == 0) bs = block_for_envs(2 * B);
    const unsigned grid = (unsigned)((2 * B + bs - 1) / bs);
#define RCBF_PAIR_L(KK, BB)                                                                                         \
    hipLaunchKernelGGL((k_uni_pair_step<KK, BB>), dim3(grid), dim3(BB), 0, stream, B, x, aux, step, u_rl, episode, \
                       obs_out, u_out, reward, cost, done, goal_met, fail_flag, auto_reset, seed, off, *prm)
#define RCBF_PAIR_K(KK)                 \
    do {                                \
        if (bs == 256)                  \
            RCBF_PAIR_L(KK, 256);       \
        else if (bs == 128)             \
            RCBF_PAIR_L(KK, 128);       \
        else                            \
            RCBF_PAIR_L(KK, 64);        \
    } while (0)
    switch (prm->num_hazards) {
        case 3:
            RCBF_PAIR_K(3);
            break;
        case 5:
            RCBF_PAIR_K(5);
            break;
        default:
            return RCBF_E_BAD_SHAPE;
    }
#undef RCBF_PAIR_K
#undef RCBF_PAIR_L
    return launch_status();
}
