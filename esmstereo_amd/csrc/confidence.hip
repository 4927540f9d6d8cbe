// Per-pixel stages of the ESMStereo confidence head (models/ESMStereo_confidence.py:511-744),
// the work between its convolutions (which run through esm_conv_f32 with ReLU / sigmoid
// epilogues).  All of it is latency-bound work on maps of 1/16 .. 1/1 of the image; every kernel
// is one thread per output pixel, all channels of the pixel in a loop, loads and stores coalesced
// along W.
//   cost features   L2normalize over D (:647-651), softmax(-100 x) (:654), topk(7).values (:655)
//   attend          softmax over the three attention logits (:679), channel-broadcast products and
//                   the concat (:681-689) in one pass
//   enlarge         the 3x grid of :691-712 built per output sample (never materialised) and
//                   F.grid_sample(bilinear, zeros, align_corners=True) (:714), stored space-to-depth
//   combine         softmax over the 9 conf_spx channels (:537), F.unfold(3,1,1) + nearest x4 (:540-
//                   541) and the weighted sum (:543)
//   sigmoid         the final torch.sigmoid (:744)
#include "common.h"

namespace esm {
namespace {

constexpr int kThreads = 256;
constexpr int kTopK = 7;
// One thread per pixel, the disparity column re-read from L1/L2 in each pass (no per-thread array:
// any D, no scratch).  Every pass recomputes -(x / nrm) * 100 with the same operations, so the values
// are those of a single pass.
__global__ void __launch_bounds__(kThreads) cost_features_kernel(const float* __restrict__ cost, float* __restrict__ out,
                                                                 int B, int D, int H, int W) {
    const long long plane = static_cast<long long>(H) * W;
    const long long i = static_cast<long long>(blockIdx.x) * kThreads + threadIdx.x;
    if (i >= B * plane) return;
    const long long b = i / plane, p = i - b * plane;
    const float* c = cost + b * D * plane + p;
    float ss = 0.f;
    for (int d = 0; d < D; ++d) {
        const float v = c[d * plane];
        ss += v * v;
    }
    // x / (sum x^2 + 1e-6) ** 0.5, then softmax(-100 * .): max, exp, sum, divide (torch order)
    const float nrm = sqrtf(ss + 1e-6f);
    float mx = -INFINITY;
    for (int d = 0; d < D; ++d) mx = fmaxf(mx, -(c[d * plane] / nrm) * 100.f);
    float se = 0.f;
    for (int d = 0; d < D; ++d) se += expf(-(c[d * plane] / nrm) * 100.f - mx);
    // top 7 of the probabilities, descending: insertion into a register list
    float top[kTopK];
#pragma unroll
    for (int k = 0; k < kTopK; ++k) top[k] = -INFINITY;
    for (int d = 0; d < D; ++d) {
        float x = expf(-(c[d * plane] / nrm) * 100.f - mx) / se;
#pragma unroll
        for (int k = 0; k < kTopK; ++k) {
            const float hi = fmaxf(top[k], x), lo = fminf(top[k], x);
            top[k] = hi;
            x = lo;
        }
    }
    float* o = out + b * kTopK * plane + p;
#pragma unroll
    for (int k = 0; k < kTopK; ++k) o[k * plane] = top[k];
}

__global__ void __launch_bounds__(kThreads) attend_kernel(const float* __restrict__ x0, const float* __restrict__ x1,
                                                          const float* __restrict__ x2, const float* __restrict__ lg,
                                                          float* __restrict__ out, int B, int C, int H, int W) {
    const long long plane = static_cast<long long>(H) * W;
    const long long i = static_cast<long long>(blockIdx.x) * kThreads + threadIdx.x;
    if (i >= B * plane) return;
    const long long b = i / plane, p = i - b * plane;
    const float l0 = lg[(b * 3 + 0) * plane + p], l1 = lg[(b * 3 + 1) * plane + p], l2 = lg[(b * 3 + 2) * plane + p];
    const float m = fmaxf(fmaxf(l0, l1), l2);
    const float e0 = expf(l0 - m), e1 = expf(l1 - m), e2 = expf(l2 - m);
    const float s = e0 + e1 + e2;
    const float a[3] = {e0 / s, e1 / s, e2 / s};
    const float* src[3] = {x0, x1, x2};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float* xs = src[k] + b * C * plane + p;
        float* o = out + (b * 3 * C + k * C) * plane + p;
        for (int c = 0; c < C; ++c) o[c * plane] = xs[c * plane] * a[k];
    }
}

// np.linspace(-1, 1, n)[i] as float32 (numpy: i * step + start in double, the last element = stop)
__device__ __forceinline__ float linspace_m11(int i, int n) {
    if (n == 1) return -1.f;
    if (i == n - 1) return 1.f;
    return static_cast<float>(static_cast<double>(i) * (2.0 / (n - 1)) - 1.0);
}

__global__ void __launch_bounds__(kThreads) enlarge_kernel(const float* __restrict__ feat, const float* __restrict__ scale,
                                                           float* __restrict__ out, int B, int C, int H, int W) {
    // one thread per (b, i, j, y, x): the sample at (3y + i, 3x + j) of the enlarged map
    const long long plane = static_cast<long long>(H) * W;
    const long long n = B * 9 * plane;
    const long long t = static_cast<long long>(blockIdx.x) * kThreads + threadIdx.x;
    if (t >= n) return;
    const long long p = t % plane;
    const int ij = static_cast<int>((t / plane) % 9);
    const long long b = t / (9 * plane);
    const int y = static_cast<int>(p / W), x = static_cast<int>(p - static_cast<long long>(y) * W);
    const int i = ij / 3, j = ij - 3 * (ij / 3);
    const float s = scale[b * plane + p];
    // grid + cat((ox * step_y * scale, oy * scale)): the python-double factor ox * step_y is
    // rounded to float before the float multiply (torch scalar-tensor arithmetic), as is oy
    // (separately rounded products and sums, as torch evaluates them: a contracted FMA here moves
    // the sample by ~(W-1)/2 ulp)
    const float fx = static_cast<float>(static_cast<double>(j - 1) * (2.0 / (W - 1)));
    const float gx = __fadd_rn(linspace_m11(x, W), __fmul_rn(fx, s));
    const float gy = __fadd_rn(linspace_m11(y, H), __fmul_rn(static_cast<float>(i - 1), s));
    // grid_sample, align_corners=True: ix = ((gx + 1) / 2) * (W - 1)
    const float ix = __fmul_rn(__fadd_rn(gx, 1.f) / 2.f, static_cast<float>(W - 1));
    const float iy = __fmul_rn(__fadd_rn(gy, 1.f) / 2.f, static_cast<float>(H - 1));
    const float fx0 = floorf(ix), fy0 = floorf(iy);
    const int x0 = static_cast<int>(fx0), y0 = static_cast<int>(fy0);
    const int x1 = x0 + 1, y1 = y0 + 1;
    const float wnw = __fmul_rn(static_cast<float>(x1) - ix, static_cast<float>(y1) - iy);
    const float wne = __fmul_rn(ix - static_cast<float>(x0), static_cast<float>(y1) - iy);
    const float wsw = __fmul_rn(static_cast<float>(x1) - ix, iy - static_cast<float>(y0));
    const float wse = __fmul_rn(ix - static_cast<float>(x0), iy - static_cast<float>(y0));
    const bool vx0 = x0 >= 0 && x0 < W, vx1 = x1 >= 0 && x1 < W, vy0 = y0 >= 0 && y0 < H, vy1 = y1 >= 0 && y1 < H;
    const float* f = feat + b * C * plane;
    float* o = out + (b * 9 * C + ij) * plane + p;
    for (int c = 0; c < C; ++c) {
        const float* fc = f + c * plane;
        float v = 0.f;  // torch accumulates nw, ne, sw, se in this order, each only when in bounds
        if (vy0 && vx0) v += fc[static_cast<long long>(y0) * W + x0] * wnw;
        if (vy0 && vx1) v += fc[static_cast<long long>(y0) * W + x1] * wne;
        if (vy1 && vx0) v += fc[static_cast<long long>(y1) * W + x0] * wsw;
        if (vy1 && vx1) v += fc[static_cast<long long>(y1) * W + x1] * wse;
        o[static_cast<long long>(c) * 9 * plane] = v;
    }
}

__global__ void __launch_bounds__(kThreads) combine_kernel(const float* __restrict__ lg, const float* __restrict__ init,
                                                           float* __restrict__ out, int B, int H, int W) {
    const int H4 = 4 * H, W4 = 4 * W;
    const long long plane4 = static_cast<long long>(H4) * W4;
    const long long t = static_cast<long long>(blockIdx.x) * kThreads + threadIdx.x;
    if (t >= B * plane4) return;
    const long long b = t / plane4, q = t - b * plane4;
    const int Y = static_cast<int>(q / W4), X = static_cast<int>(q - static_cast<long long>(Y) * W4);
    const int y = Y >> 2, x = X >> 2;
    const float* l = lg + b * 9 * plane4 + q;
    float v[9];
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        v[k] = l[k * plane4];
        m = fmaxf(m, v[k]);
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        v[k] = expf(v[k] - m);
        s += v[k];
    }
    const float* ib = init + b * static_cast<long long>(H) * W;
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
        const float u = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? ib[static_cast<long long>(yy) * W + xx] : 0.f;
        acc += u * (v[k] / s);
    }
    out[t] = acc;
}

__global__ void __launch_bounds__(kThreads) sigmoid_kernel(const float* __restrict__ x, float* __restrict__ out, long long n) {
    const long long i = static_cast<long long>(blockIdx.x) * kThreads + threadIdx.x;
    if (i < n) out[i] = 1.0f / (1.0f + expf(-x[i]));
}

}  // namespace

int launch_conf(const esm_conf_desc* d, hipStream_t s) {
    if (!d) return arg_error("conf: null descriptor");
    const esm_conf_desc& a = *d;
    if (a.B <= 0 || a.H <= 0 || a.W <= 0) return arg_error("conf: bad size");
    if (!a.out || !a.x[0]) return arg_error("conf: null pointer");
    const long long px = static_cast<long long>(a.B) * a.H * a.W;
    switch (a.op) {
        case ESM_CONF_COST_FEATURES:
            if (a.D < kTopK) return arg_error("conf: cost features need D >= 7 (torch.topk(7))");
            hipLaunchKernelGGL(cost_features_kernel, dim3(ceil_div(px, kThreads)), dim3(kThreads), 0, s, a.x[0], a.out,
                               a.B, a.D, a.H, a.W);
            break;
        case ESM_CONF_ATTEND:
            if (!a.x[1] || !a.x[2] || !a.x[3] || a.C <= 0) return arg_error("conf: attend needs x[0..3] and C > 0");
            hipLaunchKernelGGL(attend_kernel, dim3(ceil_div(px, kThreads)), dim3(kThreads), 0, s, a.x[0], a.x[1], a.x[2],
                               a.x[3], a.out, a.B, a.C, a.H, a.W);
            break;
        case ESM_CONF_ENLARGE:
            if (!a.x[1] || a.C <= 0 || a.H < 2 || a.W < 2) return arg_error("conf: enlarge needs scale, C > 0, H, W >= 2");
            hipLaunchKernelGGL(enlarge_kernel, dim3(ceil_div(9 * px, kThreads)), dim3(kThreads), 0, s, a.x[0], a.x[1],
                               a.out, a.B, a.C, a.H, a.W);
            break;
        case ESM_CONF_COMBINE:
            if (!a.x[1]) return arg_error("conf: combine needs init");
            hipLaunchKernelGGL(combine_kernel, dim3(ceil_div(16 * px, kThreads)), dim3(kThreads), 0, s, a.x[0], a.x[1],
                               a.out, a.B, a.H, a.W);
            break;
        case ESM_CONF_SIGMOID: {
            const long long n = px * (a.C > 0 ? a.C : 1);
            hipLaunchKernelGGL(sigmoid_kernel, dim3(ceil_div(n, kThreads)), dim3(kThreads), 0, s, a.x[0], a.out, n);
            break;
        }
        default: return arg_error("conf: unknown op");
    }
    return check_launch("conf");
}

}  // namespace esm

extern "C" int esm_conf_f32(const esm_conf_desc* desc, void* stream) {
    return esm::launch_conf(desc, esm::as_stream(stream));
}
