// Probe: workgroup dispatch cost on gfx950 — empty-ish 256-thread workgroups, by grid size,
// with a small kernel argument and with a ~400-byte by-value struct (the size of esm_conv_desc).
#include <hip/hip_runtime.h>
#include <cstdio>

struct Big {
    float* out;
    int v[100];
};

__global__ void __launch_bounds__(256) small_k(float* out, int n) {
    if (threadIdx.x == 0 && blockIdx.x == 0xffffffffu) out[0] = n;
}

__global__ void __launch_bounds__(256) big_k(const Big b) {
    if (threadIdx.x == 0 && blockIdx.x == 0xffffffffu) b.out[0] = b.v[blockIdx.x % 100];
}

// reads ~all of the struct (as the conv kernels do) before a trivial store
__global__ void __launch_bounds__(256) big_read_k(const Big b) {
    int s = 0;
#pragma unroll
    for (int i = 0; i < 100; ++i) s += b.v[i];
    if (s == 123456789 && threadIdx.x == 0) b.out[0] = s;
}

template <typename F>
float time_it(F launch, int reps) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    launch();
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < reps; ++i) launch();
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms * 1e3f / reps;
}

int main() {
    float* out;
    if (hipMalloc(&out, 64) != hipSuccess) return 1;
    Big b{};
    b.out = out;
    printf("%8s %10s %10s %10s  (us per launch, stream-ordered)\n", "WGs", "small", "big", "big+read");
    for (int n : {1, 256, 1024, 2048, 4096, 8192, 16384}) {
        const float ts = time_it([&] { hipLaunchKernelGGL(small_k, dim3(n), dim3(256), 0, 0, out, n); }, 50);
        const float tb = time_it([&] { hipLaunchKernelGGL(big_k, dim3(n), dim3(256), 0, 0, b); }, 50);
        const float tr = time_it([&] { hipLaunchKernelGGL(big_read_k, dim3(n), dim3(256), 0, 0, b); }, 50);
        printf("%8d %10.2f %10.2f %10.2f\n", n, ts, tb, tr);
    }
    return 0;
}
