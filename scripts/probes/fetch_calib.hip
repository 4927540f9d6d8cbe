// Calibration of the FETCH_SIZE / WRITE_SIZE counters for the access widths our kernels use
// (MI355X_MICROARCH.md §HBM: only 16-B/lane streaming reads and writes are calibrated there).
// Each kernel touches every byte of a 64 MiB buffer exactly once, coalesced, at one width; run under
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib      and      rocprofv3 --pmc WRITE_SIZE -- ./fetch_calib
// and divide the per-dispatch counter (KiB) by the bytes below.  Plain global loads / stores here;
// the buffer_load forms of the kernels move the same cache lines.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr size_t kBytes = 64ull << 20;

template <int V>
__global__ void __launch_bounds__(256) read_k(const float* __restrict__ x, float* __restrict__ sink) {
    const size_t i = (static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x) * V;
    float s = 0.f;
    if constexpr (V == 1) s = x[i];
    if constexpr (V == 2) {
        const float2 v = *reinterpret_cast<const float2*>(x + i);
        s = v.x + v.y;
    }
    if constexpr (V == 4) {
        const float4 v = *reinterpret_cast<const float4*>(x + i);
        s = v.x + v.y + v.z + v.w;
    }
    if (s == 12345.678f) sink[0] = s;  // never true for the zero-filled input: keeps the loads alive
}

// Row segments of 10 floats at float offset 32k + 31 of rows 1248 floats apart (k = 0..37): each
// segment crosses a 128-B line boundary, the shape of a shuffle_tail low-resolution window row.  The
// counter over the requested bytes (rows * 38 * 40) gives the fetch granularity of such rows.
__global__ void __launch_bounds__(256) read_window(const float* __restrict__ x, float* __restrict__ sink, int rows) {
    const int t = threadIdx.x;
    const int seg = blockIdx.x * 25 + t / 10;  // 25 segments of 10 floats per block (250 lanes)
    if (t >= 250 || seg >= rows * 38) return;
    const int row = seg / 38, k = seg % 38;
    const float v = x[static_cast<size_t>(row) * 1248 + 32 * k + 31 + t % 10];
    if (v == 12345.678f) sink[0] = v;
}

template <int V>
__global__ void __launch_bounds__(256) write_k(float* __restrict__ y) {
    const size_t i = (static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x) * V;
    if constexpr (V == 1) y[i] = 1.f;
    if constexpr (V == 4) *reinterpret_cast<float4*>(y + i) = float4{1.f, 1.f, 1.f, 1.f};
}

int main() {
    float *x = nullptr, *y = nullptr, *sink = nullptr;
    if (hipMalloc(&x, kBytes) != hipSuccess || hipMalloc(&y, kBytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess)
        return 1;
    hipMemset(x, 0, kBytes);
    hipMemset(y, 0, kBytes);
    const size_t n = kBytes / 4;
    for (int rep = 0; rep < 3; ++rep) {
        // reads of x at 4 / 8 / 16 B per lane and in row windows, writes of y at 16 / 4 B per lane
        hipLaunchKernelGGL((read_k<1>), dim3(n / 256), dim3(256), 0, 0, x, sink);
        hipLaunchKernelGGL((write_k<4>), dim3(n / 1024), dim3(256), 0, 0, y);
        hipLaunchKernelGGL((read_k<2>), dim3(n / 512), dim3(256), 0, 0, x, sink);
        hipLaunchKernelGGL((write_k<4>), dim3(n / 1024), dim3(256), 0, 0, y);
        hipLaunchKernelGGL((read_k<4>), dim3(n / 1024), dim3(256), 0, 0, x, sink);
        hipLaunchKernelGGL((write_k<1>), dim3(n / 256), dim3(256), 0, 0, y);
        const int rows = static_cast<int>(n / 1248);
        hipLaunchKernelGGL(read_window, dim3((rows * 38 + 24) / 25), dim3(256), 0, 0, x, sink, rows);
        hipLaunchKernelGGL((write_k<4>), dim3(n / 1024), dim3(256), 0, 0, y);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    const int rows = static_cast<int>(n / 1248);
    std::printf("bytes per read_k / write_k dispatch: %zu; read_window requested bytes: %lld\n", kBytes,
                static_cast<long long>(rows) * 38 * 10 * 4);
    hipFree(x);
    hipFree(y);
    hipFree(sink);
    return 0;
}
