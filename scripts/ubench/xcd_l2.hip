// Micro-benchmark (diagnostic, not product): is the workgroup -> XCD
// placement the same from one launch to the next, and does a chunk that a
// workgroup stored in launch k come back from its XCD's L2 in launch k+1?
// Mimics the fused step's access shape: 256 workgroups x 256 lanes, each lane
// loads 5 x 16 B + stores 5 x 16 B of its own chunk per launch.
// Build: hipcc --offload-arch=gfx950 -O3 -o xcd_l2 xcd_l2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_ids(int* ids) {
    if (threadIdx.x == 0) {
        unsigned v;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
        ids[blockIdx.x] = (int)(v & 0xf);
    }
}

// chunk = (blockIdx.x + shift) % nblk; NT selects nt loads/stores
template <bool NT>
__global__ void k_rw(double* x, int nblk, int shift, int64_t B) {
    if ((int)blockIdx.x >= nblk) return;  // grid padded to a multiple of 8 workgroups
    const int chunk = (blockIdx.x + shift) % nblk;
    const int64_t i = (int64_t)chunk * blockDim.x + threadIdx.x;
    typedef double d2 __attribute__((ext_vector_type(2)));
    d2 v[5];
#pragma unroll
    for (int p = 0; p < 5; ++p) {
        d2* a = reinterpret_cast<d2*>(x + 2 * (p * B + i));
        v[p] = NT ? __builtin_nontemporal_load(a) : *a;
    }
#pragma unroll
    for (int p = 0; p < 5; ++p) {
        v[p].x = v[p].x * 1.0000001 + 1e-9;
        v[p].y = v[p].y * 0.9999999 - 1e-9;
    }
#pragma unroll
    for (int p = 0; p < 5; ++p) {
        d2* a = reinterpret_cast<d2*>(x + 2 * (p * B + i));
        if (NT)
            __builtin_nontemporal_store(v[p], a);
        else
            *a = v[p];
    }
}

int main() {
    const int nblk = 256, T = 256;
    const int64_t B = (int64_t)nblk * T;
    int* ids;
    hipMalloc(&ids, nblk * sizeof(int));
    std::vector<int> h0(nblk), h1(nblk);
    int same_total = 0, launches = 20;
    for (int l = 0; l < launches; ++l) {
        hipLaunchKernelGGL(k_ids, dim3(nblk), dim3(T), 0, 0, ids);
        hipMemcpy(l ? h1.data() : h0.data(), ids, nblk * sizeof(int), hipMemcpyDeviceToHost);
        if (l) {
            int same = 0;
            for (int b = 0; b < nblk; ++b) same += h0[b] == h1[b];
            same_total += same;
            if (l < 4) printf("launch %d: %d/%d workgroups on the same XCC as launch 0 (b0 -> xcc %d, b1 -> %d)\n", l,
                              same, nblk, h1[0], h1[1]);
        }
    }
    printf("mean same-XCC fraction over %d launches: %.3f\n", launches - 1,
           same_total / double(nblk * (launches - 1)));
    // back-to-back (no host sync between) launches: placement in a stream
    double* x;
    hipMalloc(&x, 10 * B * sizeof(double));
    hipMemset(x, 0, 10 * B * sizeof(double));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int reps = 2000;
    // grid = nblk workgroups, or nblk rounded up to a multiple of 8 (the extra ones exit at once)
    for (int nb : {256, 260, 260, 255}) {
        for (int pad = 0; pad < 2; ++pad) {
            const int grid = pad ? (nb + 7) / 8 * 8 : nb;
            for (int shift : {0, 1}) {
                for (int r = 0; r < 50; ++r)
                    hipLaunchKernelGGL(k_rw<true>, dim3(grid), dim3(T), 0, 0, x, nb, (r & 1) ? shift : 0, B);
                hipEventRecord(e0, 0);
                for (int r = 0; r < reps; ++r)
                    hipLaunchKernelGGL(k_rw<true>, dim3(grid), dim3(T), 0, 0, x, nb, (r & 1) ? shift : 0, B);
                hipEventRecord(e1, 0);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                printf("nt %d chunks on %d workgroups, shift %d: %.3f us per launch\n", nb, grid, shift, ms * 1e3 / reps);
            }
        }
    }
    hipFree(x);
    hipFree(ids);
    return 0;
}
