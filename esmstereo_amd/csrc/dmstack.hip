// The ESM upsamplers' disparity-feature stack `dm<tag>` (models/ESMStereo.py:250-253, used :292,
// :374, :466): four BasicConv2d (conv bias=False -> BN -> exact GELU, models/submodule.py:12-38)
//   L0 k5 p1  1 -> C   (H x W -> H-2 x W-2)
//   L1 k3 p1  C -> C
//   L2 k3 p1  C -> C
//   L3 k1 p1  C -> C   (H-2 x W-2 -> H x W; the ring is GELU(BN(0)) = GELU(shift))
// in one launch with halo recomputation, instead of four launches whose chain is latency-bound on
// the 1/16 .. 1/4 resolution maps.  "d-space" is the H-2 x W-2 grid of L0..L2.  A workgroup owns a
// TH x TW d-space tile: it stages the single-channel input under the tile plus a 4-pixel halo,
// computes L0 on the tile plus 2, L1 on the tile plus 1 (each zero outside d-space: the next conv's
// zero padding), L2 on the tile, and writes L3 for its tile shifted by one (plus the ring, for
// workgroups on the map's border).
// Work split: a wave owns C / 8 output channels (wave-uniform, so every weight and BN value is a
// scalar load), a lane one pixel; each activation read from LDS feeds all of the wave's channels.
#include "common.h"

namespace esm {
namespace {

constexpr int kDThreads = 512;
constexpr int kDWaves = kDThreads / 64;

template <int C, int TH, int TW>
__global__ void __launch_bounds__(kDThreads) dmstack_kernel(const esm_dmstack_desc a) {
    constexpr int CPW = C / kDWaves;                  // output channels per wave
    constexpr int R0H = TH + 4, R0W = TW + 4;         // L0 region (d-space origin: tile - 2)
    constexpr int R1H = TH + 2, R1W = TW + 2;         // L1 region (tile - 1)
    constexpr int IH = TH + 8, IW = TW + 8;           // input region (input origin: tile - 3)
    constexpr int FH = TH + 2, FW = TW + 2;           // largest output region (with the ring)
    static_assert(C % kDWaves == 0, "C / 8 channels per wave");
    __shared__ float sin_[IH * IW];
    __shared__ float s0[C * R0H * R0W];
    __shared__ float s1[C * R1H * R1W];
    __shared__ float s2[C * TH * TW];
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid / 64), lane = tid % 64;
    const int H = a.H, W = a.W, Hd = H - 2, Wd = W - 2;
    const int b = blockIdx.z;
    const int ya = blockIdx.y * TH, xa = blockIdx.x * TW;
    const int co0 = wave * CPW;
    const float* xin = a.x + static_cast<long long>(b) * a.xb;

    for (int i = tid; i < IH * IW; i += kDThreads) {
        const int r = i / IW, c = i - (i / IW) * IW;
        const int gy = ya - 3 + r, gx = xa - 3 + c;
        const bool ok = gy >= 0 && gy < H && gx >= 0 && gx < W;
        const float v = xin[ok ? static_cast<long long>(gy) * a.xh + gx : 0];
        sin_[i] = ok ? v : 0.f;
    }
    __syncthreads();
    // L0: 5x5, 1 -> C on the tile + 2
    for (int p = lane; p < R0H * R0W; p += 64) {
        const int ry = p / R0W, rx = p - (p / R0W) * R0W;
        const int gy = ya - 2 + ry, gx = xa - 2 + rx;
        const bool in = gy >= 0 && gy < Hd && gx >= 0 && gx < Wd;
        float acc[CPW];
#pragma unroll
        for (int j = 0; j < CPW; ++j) acc[j] = 0.f;
#pragma unroll
        for (int ky = 0; ky < 5; ++ky)
#pragma unroll
            for (int kx = 0; kx < 5; ++kx) {
                const float v = sin_[(ry + ky) * IW + rx + kx];
#pragma unroll
                for (int j = 0; j < CPW; ++j) acc[j] += a.w[0][(co0 + j) * 25 + ky * 5 + kx] * v;
            }
#pragma unroll
        for (int j = 0; j < CPW; ++j)
            s0[((co0 + j) * R0H + ry) * R0W + rx] =
                in ? gelu_erf(acc[j] * a.scale[0][co0 + j] + a.shift[0][co0 + j]) : 0.f;
    }
    __syncthreads();
    // L1: 3x3, C -> C on the tile + 1
    for (int p = lane; p < R1H * R1W; p += 64) {
        const int ry = p / R1W, rx = p - (p / R1W) * R1W;
        const int gy = ya - 1 + ry, gx = xa - 1 + rx;
        const bool in = gy >= 0 && gy < Hd && gx >= 0 && gx < Wd;
        float acc[CPW];
#pragma unroll
        for (int j = 0; j < CPW; ++j) acc[j] = 0.f;
#pragma unroll
        for (int ci = 0; ci < C; ++ci)
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    const float v = s0[(ci * R0H + ry + ky) * R0W + rx + kx];
#pragma unroll
                    for (int j = 0; j < CPW; ++j) acc[j] += a.w[1][((co0 + j) * C + ci) * 9 + ky * 3 + kx] * v;
                }
#pragma unroll
        for (int j = 0; j < CPW; ++j)
            s1[((co0 + j) * R1H + ry) * R1W + rx] =
                in ? gelu_erf(acc[j] * a.scale[1][co0 + j] + a.shift[1][co0 + j]) : 0.f;
    }
    __syncthreads();
    // L2: 3x3, C -> C on the tile (positions past d-space are computed but never read)
    for (int p = lane; p < TH * TW; p += 64) {
        const int ry = p / TW, rx = p - (p / TW) * TW;
        float acc[CPW];
#pragma unroll
        for (int j = 0; j < CPW; ++j) acc[j] = 0.f;
#pragma unroll
        for (int ci = 0; ci < C; ++ci)
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    const float v = s1[(ci * R1H + ry + ky) * R1W + rx + kx];
#pragma unroll
                    for (int j = 0; j < CPW; ++j) acc[j] += a.w[2][((co0 + j) * C + ci) * 9 + ky * 3 + kx] * v;
                }
#pragma unroll
        for (int j = 0; j < CPW; ++j)
            s2[((co0 + j) * TH + ry) * TW + rx] = gelu_erf(acc[j] * a.scale[2][co0 + j] + a.shift[2][co0 + j]);
    }
    __syncthreads();
    // L3: 1x1 with padding 1 -> the H x W output.  Output (y, x) with 1 <= y < H-1 reads L2 at
    // d-space (y-1, x-1); this workgroup writes rows ya+1 .. ya+TH (plus row 0 / the rows up to H-1
    // when its tile touches that edge), and the same for columns.
    const int ylo = blockIdx.y == 0 ? 0 : ya + 1;
    const int yhi = ya + TH >= Hd ? H : ya + TH + 1;
    const int xlo = blockIdx.x == 0 ? 0 : xa + 1;
    const int xhi = xa + TW >= Wd ? W : xa + TW + 1;
    const int fw = xhi - xlo, nf = (yhi - ylo) * fw;
    float* ob = a.out + static_cast<long long>(b) * C * H * W;
    for (int p = lane; p < nf && p < FH * FW; p += 64) {
        const int y = ylo + p / fw, x = xlo + p - (p / fw) * fw;
        const bool ring = y == 0 || y == H - 1 || x == 0 || x == W - 1;
        float acc[CPW];
#pragma unroll
        for (int j = 0; j < CPW; ++j) acc[j] = 0.f;
        if (!ring) {
            const int ry = y - 1 - ya, rx = x - 1 - xa;
#pragma unroll
            for (int ci = 0; ci < C; ++ci) {
                const float v = s2[(ci * TH + ry) * TW + rx];
#pragma unroll
                for (int j = 0; j < CPW; ++j) acc[j] += a.w[3][(co0 + j) * C + ci] * v;
            }
        }
#pragma unroll
        for (int j = 0; j < CPW; ++j)
            ob[(static_cast<long long>(co0 + j) * H + y) * W + x] =
                gelu_erf(acc[j] * a.scale[3][co0 + j] + a.shift[3][co0 + j]);
    }
}

}  // namespace

int launch_dmstack(const esm_dmstack_desc* d, hipStream_t s) {
    if (!d) return arg_error("dmstack: null descriptor");
    const esm_dmstack_desc& a = *d;
    if (!a.x || !a.out) return arg_error("dmstack: null pointer");
    for (int l = 0; l < 4; ++l)
        if (!a.w[l] || !a.scale[l] || !a.shift[l]) return arg_error("dmstack: null weight / BN pointer");
    if (a.B <= 0 || a.H < 3 || a.W < 3) return arg_error("dmstack: needs B >= 1 and H, W >= 3 (k5 p1)");
    if (a.xb < static_cast<int64_t>(a.H) * a.xh || a.xh < a.W) return arg_error("dmstack: bad input strides");
    if (a.C != 16) {
        set_error("dmstack: C must be 16");
        return ESM_ERR_UNSUPPORTED;
    }
    constexpr int TH = 4, TW = 8;
    const dim3 grid(ceil_div(a.W - 2, TW), ceil_div(a.H - 2, TH), a.B);
    hipLaunchKernelGGL((dmstack_kernel<16, TH, TW>), grid, dim3(kDThreads), 0, s, a);
    return check_launch("dmstack");
}

}  // namespace esm

extern "C" int esm_dmstack_f32(const esm_dmstack_desc* desc, void* stream) {
    return esm::launch_dmstack(desc, esm::as_stream(stream));
}
