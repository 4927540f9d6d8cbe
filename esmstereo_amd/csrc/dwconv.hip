// Depthwise KxK convolution + folded BatchNorm + activation: the `conv_dw -> bn` of timm's
// DepthwiseSeparableConv / InvertedResidual blocks (the backbone side of the forward,
// models/ESMStereo.py:40-77; esmstereo_amd/backbone.py restates the blocks).
// PyTorch-ROCm runs these grouped convs through MIOpen's naive direct kernel (55 us a launch at
// 192 x 624, the largest share of the backbone's device time); here they are one HBM-bound pass.
//
// A workgroup (256 threads) owns a TY x TX output tile of one (batch, channel) plane: it stages the
// input window (TY*s + K - 1) x (TX*s + K - 1) in LDS with coalesced loads (zero outside the image:
// the conv's zero padding), then every thread computes NX consecutive outputs of one row from LDS,
// the K*K weights and the BN pair wave-uniform (scalar loads).  Per output the products are summed
// over ky, then kx (fp32, the tolerance of tests/test_gpu_backbone.py vs the PyTorch module).
#include "common.h"

namespace esm {
namespace {

constexpr int kDwThreads = 256;
constexpr int kDwTX = 64, kDwTY = 8, kDwNX = kDwTX * kDwTY / kDwThreads;  // 2 outputs a thread

template <int K, int S>
__global__ void __launch_bounds__(kDwThreads) dwconv_kernel(const esm_dwconv_desc a) {
    constexpr int IW = kDwTX * S + K - 1, IH = kDwTY * S + K - 1;
    constexpr int IWP = IW + 1;
    __shared__ float tile[IH * IWP];
    const int tid = threadIdx.x;
    // grid x = (b * C + c) * tiles_x + tile x (planes on x: the z grid's 65535 limit is below B * C of the
    // backbone's [left; right] batch at configs[3]'s 32 pairs)
    const int ntx = (a.Wo + kDwTX - 1) / kDwTX;
    const int plane = blockIdx.x / ntx;
    const int b = plane / a.C, c = plane - (plane / a.C) * a.C;
    const int oy0 = blockIdx.y * kDwTY, ox0 = (blockIdx.x - plane * ntx) * kDwTX;
    const int iy0 = oy0 * S - a.pad, ix0 = ox0 * S - a.pad;
    const float* xp = a.x + b * a.xb + c * a.xc;
    for (int i = tid; i < IH * IW; i += kDwThreads) {
        const int r = i / IW, q = i - (i / IW) * IW;
        const int y = iy0 + r, x = ix0 + q;
        const bool ok = y >= 0 && y < a.H && x >= 0 && x < a.W;
        const float v = xp[ok ? static_cast<long long>(y) * a.xh + x : 0];
        tile[r * IWP + q] = ok ? v : 0.f;
    }
    float w[K * K];
#pragma unroll
    for (int i = 0; i < K * K; ++i) w[i] = a.w[c * K * K + i];
    const float sc = a.scale ? a.scale[c] : 1.f, sh = a.shift ? a.shift[c] : 0.f;
    __syncthreads();
    const int ty = tid / (kDwTX / kDwNX), tx = (tid - ty * (kDwTX / kDwNX)) * kDwNX;
    const int oy = oy0 + ty;
    if (oy >= a.Ho) return;
    float acc[kDwNX];
#pragma unroll
    for (int j = 0; j < kDwNX; ++j) acc[j] = 0.f;
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
        const float* row = &tile[(ty * S + ky) * IWP + tx * S];
        float v[(kDwNX - 1) * S + K];
#pragma unroll
        for (int j = 0; j < (kDwNX - 1) * S + K; ++j) v[j] = row[j];
#pragma unroll
        for (int kx = 0; kx < K; ++kx)
#pragma unroll
            for (int j = 0; j < kDwNX; ++j) acc[j] += w[ky * K + kx] * v[j * S + kx];
    }
    float* op = a.out + b * a.ob + c * a.oc + static_cast<long long>(oy) * a.oh;
#pragma unroll
    for (int j = 0; j < kDwNX; ++j)
        if (ox0 + tx + j < a.Wo) op[ox0 + tx + j] = apply_act(acc[j] * sc + sh, a.act);
}

template <int K, int S>
int launch_dw(const esm_dwconv_desc& a, hipStream_t s) {
    const dim3 grid(static_cast<unsigned>(ceil_div(a.Wo, kDwTX) * a.B * a.C), ceil_div(a.Ho, kDwTY), 1);
    hipLaunchKernelGGL((dwconv_kernel<K, S>), grid, dim3(kDwThreads), 0, s, a);
    return check_launch("dwconv");
}

}  // namespace

int launch_dwconv(const esm_dwconv_desc* d, hipStream_t s) {
    if (!d) return arg_error("dwconv: null descriptor");
    const esm_dwconv_desc& a = *d;
    if (!a.x || !a.w || !a.out) return arg_error("dwconv: null pointer");
    if (a.B <= 0 || a.C <= 0 || a.H <= 0 || a.W <= 0) return arg_error("dwconv: bad size");
    if (a.stride <= 0 || a.K <= 0) return arg_error("dwconv: stride and K must be positive");
    if (a.pad < 0 || a.pad >= a.K) return arg_error("dwconv: bad padding");
    if (a.Ho != (a.H + 2 * a.pad - a.K) / a.stride + 1 || a.Wo != (a.W + 2 * a.pad - a.K) / a.stride + 1 || a.Ho <= 0 ||
        a.Wo <= 0)
        return arg_error("dwconv: output extent inconsistent with K / stride / pad");
    if (a.xh < a.W || a.xc < static_cast<long long>(a.H) * a.xh || a.oh < a.Wo || a.oc < static_cast<long long>(a.Ho) * a.oh)
        return arg_error("dwconv: strides inconsistent with the extents");
    if (static_cast<long long>(ceil_div(a.Wo, kDwTX)) * a.B * a.C > 0x7fffffffLL || ceil_div(a.Ho, kDwTY) > 65535u)
        return arg_error("dwconv: grid too large");  // (grid x / y limits)
    if (a.K == 3 && a.stride == 1) return launch_dw<3, 1>(a, s);
    if (a.K == 3 && a.stride == 2) return launch_dw<3, 2>(a, s);
    if (a.K == 5 && a.stride == 1) return launch_dw<5, 1>(a, s);
    if (a.K == 5 && a.stride == 2) return launch_dw<5, 2>(a, s);
    set_error("dwconv: (K, stride) must be one of (3, 1), (3, 2), (5, 1), (5, 2)");
    return ESM_ERR_UNSUPPORTED;
}

}  // namespace esm

extern "C" int esm_dwconv_f32(const esm_dwconv_desc* desc, void* stream) {
    return esm::launch_dwconv(desc, esm::as_stream(stream));
}
