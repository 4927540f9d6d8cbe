// Probe: what does a kernel's code size cost a latency-bound launch?  Kernels of N dependent FMAs,
// straight-line (code ~8 B x N) or as a short loop (same work, ~100 B of code), launched as a
// dependent chain on one stream:
//   (a) the same kernel back to back (its code warm in the instruction caches),
//   (b) 16 distinct instantiations in rotation (each launch finds the per-CU instruction cache
//       holding other code; L2 warm),
//   (c) (b) with a 64 MB copy between launches (L2 flushed of the code too; copy time subtracted).
//   hipcc -O3 --offload-arch=gfx950 -o scripts/probes/icache_probe scripts/probes/icache_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

template <int N, int SALT, bool LOOP>
__global__ void __launch_bounds__(256) chain(float* out, float a) {
    float x = static_cast<float>(threadIdx.x) + SALT;
    if constexpr (LOOP) {
        // a 64-FMA body (~512 B of code) run N / 64 times: the same dependent chain from a hot loop
#pragma unroll 1
        for (int j = 0; j < N / 64; ++j)
#pragma unroll
            for (int i = 0; i < 64; ++i) x = __builtin_fmaf(x, a, 0.5f * i + SALT);
    } else {
#pragma unroll
        for (int i = 0; i < N; ++i) x = __builtin_fmaf(x, a, 0.5f * i + SALT);
    }
    out[blockIdx.x * 256 + threadIdx.x] = x;
}

__global__ void copyk(const float4* __restrict__ s, float4* __restrict__ d, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * 256) d[i] = s[i];
}

using KFn = void (*)(float*, float);

template <int N, bool LOOP, int... S>
void table(KFn* k, std::integer_sequence<int, S...>) {
    ((k[S] = chain<N, S, LOOP>), ...);
}

template <typename F>
float timeit(F f, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 16; ++i) f(i);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    for (int i = 0; i < reps; ++i) f(i);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / reps * 1e3f;
}

float* g_out;
float4 *g_s, *g_d;
const size_t kCopy = (64u << 20) / 16;

template <int N, bool LOOP>
void run(int grid) {
    KFn k[16];
    table<N, LOOP>(k, std::make_integer_sequence<int, 16>{});
    const float same = timeit([&](int) { hipLaunchKernelGGL(k[0], dim3(grid), dim3(256), 0, 0, g_out, 1.0001f); }, 400);
    const float rot = timeit([&](int i) { hipLaunchKernelGGL(k[i % 16], dim3(grid), dim3(256), 0, 0, g_out, 1.0001f); }, 400);
    const float cp = timeit([&](int) { hipLaunchKernelGGL(copyk, dim3(1024), dim3(256), 0, 0, g_s, g_d, kCopy); }, 100);
    const float rotc = timeit([&](int i) {
        hipLaunchKernelGGL(copyk, dim3(1024), dim3(256), 0, 0, g_s, g_d, kCopy);
        hipLaunchKernelGGL(k[i % 16], dim3(grid), dim3(256), 0, 0, g_out, 1.0001f);
    }, 100);
    printf("N %5d %-8s grid %4d: same %6.2f us | rotating 16 %6.2f us | after 64MB copy %6.2f us (copy %6.2f)\n", N,
           LOOP ? "loop" : "straight", grid, same, rot, rotc - cp, cp);
}

int main() {
    (void)hipMalloc(&g_out, 4 << 20);
    (void)hipMalloc(&g_s, kCopy * 16);
    (void)hipMalloc(&g_d, kCopy * 16);
    for (int grid : {256, 2048}) {
        run<8, false>(grid);
        run<512, false>(grid);
        run<512, true>(grid);
        run<1024, false>(grid);
        run<1024, true>(grid);
        run<2048, false>(grid);
        run<2048, true>(grid);
        run<4096, false>(grid);
        run<4096, true>(grid);
    }
    return 0;
}
