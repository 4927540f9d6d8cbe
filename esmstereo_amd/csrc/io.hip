// The steps on either side of the hot path, as HBM-bound elementwise
// kernels on device-resident images:
//
//  esm_preprocess_u8  8-bit RGB [B, H, W, 3] -> ImageNet-normalised [B, 3, Hp, Wp] fp32, padded:
//    pad_normalized = 1: test_kitti.py:93-106 — PIL crop (w - wi, h - hi, w, h) pads the uint8
//      image with zeros at the top-left, THEN ToTensor + Normalize, so the padding holds
//      (0 - mean) / std;
//    pad_normalized = 0: datasets/kitti_dataset.py:151-170 — ToTensor + Normalize, THEN np.pad
//      with 0.0 at the top and right.
//    Value: ((float)u8 / 255 - mean[c]) / std[c], each operation rounded in fp32 as torchvision's
//    to_tensor (`.div(255)`) and Normalize (`sub_(mean).div_(std)`, fp32 mean/std) do
//    (datasets/data_io.py:7-16): bit-exact.
//  esm_disp_to_u16    disparity [B, Hp, Wp] fp32 -> KITTI 16-bit PNG values [B, h, w]:
//    window (top, left, h, w) of the padded map (test_kitti.py:115 `pred[:, hi-h:, wi-w:]`,
//    save_disp.py:81 `disp[top_pad:, :-right_pad]`), then np.round(d * 256).astype(np.uint16)
//    (save_disp.py:85): round half to even (rintf), then the low 16 bits of the integer (numpy's
//    float -> uint16 cast on x86-64 goes through a 32-bit integer; a disparity in [0, 256) -
//    every KITTI value - is exact either way).
//  esm_node_filter_u16  the ROS node's post-processing (kitti_publisher_cuda_node.cpp:385-397) on the
//    device: crop to the image (:385-388), cv::medianBlur 5x5 (BORDER_REPLICATE inside the crop,
//    :391), valid_mask = (d > 0) & (d < max_disp) with the rest set to 0 (:400-402),
//    convertTo(CV_16UC1, 256.0) = saturate_cast<ushort>(rint(d * 256)) (:403).
// One thread per output element, consecutive threads along W (coalesced 4-byte stores); the
// RGB reads are 3-byte strided and served by L1/L2 (each 64-lane load touches 192 contiguous bytes).
#include "common.h"

// one rounding per torchvision operation
#pragma clang fp contract(off)

namespace esm {
namespace {

constexpr int kThreads = 256;

__global__ void __launch_bounds__(kThreads) preprocess_kernel(const uint8_t* __restrict__ img, float* __restrict__ out,
                                                              int H, int W, int Hp, int Wp, int top, int left,
                                                              int pad_normalized, long long n) {
    const long long i = static_cast<long long>(blockIdx.x) * kThreads + threadIdx.x;
    if (i >= n) return;
    const int x = static_cast<int>(i % Wp);
    long long t = i / Wp;
    const int y = static_cast<int>(t % Hp);
    t /= Hp;
    const int c = static_cast<int>(t % 3);
    const long long b = t / 3;
    // torchvision Normalize constants as fp32 tensors (datasets/data_io.py:8-9)
    const float mean = c == 0 ? 0.485f : (c == 1 ? 0.456f : 0.406f);
    const float stdv = c == 0 ? 0.229f : (c == 1 ? 0.224f : 0.225f);
    const int sy = y - top, sx = x - left;
    const bool inside = sy >= 0 && sy < H && sx >= 0 && sx < W;
    float v;
    if (inside) {
        const float u = static_cast<float>(img[((b * H + sy) * W + sx) * 3 + c]);
        v = (u / 255.0f - mean) / stdv;
    } else {
        v = pad_normalized ? (0.0f / 255.0f - mean) / stdv : 0.0f;
    }
    out[i] = v;
}

__global__ void __launch_bounds__(kThreads) disp_u16_kernel(const float* __restrict__ disp, uint16_t* __restrict__ out,
                                                            int Hp, int Wp, int top, int left, int h, int w,
                                                            long long n) {
    const long long i = static_cast<long long>(blockIdx.x) * kThreads + threadIdx.x;
    if (i >= n) return;
    const int x = static_cast<int>(i % w);
    long long t = i / w;
    const int y = static_cast<int>(t % h);
    const long long b = t / h;
    const float d = disp[(b * Hp + (y + top)) * Wp + (x + left)];
    const float r = rintf(d * 256.0f);
    out[i] = static_cast<uint16_t>(static_cast<uint32_t>(static_cast<int32_t>(r)));
}

// median of 25 by a full compare-exchange sort (exact: selection only, no arithmetic)
__device__ __forceinline__ float median25(float (&v)[25]) {
#pragma unroll
    for (int i = 0; i < 25; ++i)
#pragma unroll
        for (int j = 0; j < 24 - i; ++j) {
            const float a = v[j], b = v[j + 1];
            v[j] = fminf(a, b);
            v[j + 1] = fmaxf(a, b);
        }
    return v[12];
}

__global__ void __launch_bounds__(kThreads) node_filter_kernel(const float* __restrict__ disp, uint16_t* __restrict__ out,
                                                               float* __restrict__ filtered, int Hp, int Wp, int top,
                                                               int left, int h, int w, float max_disp, long long n) {
    const long long i = static_cast<long long>(blockIdx.x) * kThreads + threadIdx.x;
    if (i >= n) return;
    const int x = static_cast<int>(i % w);
    long long t = i / w;
    const int y = static_cast<int>(t % h);
    const long long b = t / h;
    const float* d = disp + (b * Hp + top) * Wp + left;
    float v[25];
#pragma unroll
    for (int dy = 0; dy < 5; ++dy) {
        const int yy = min(max(y + dy - 2, 0), h - 1);  // BORDER_REPLICATE inside the cropped window
#pragma unroll
        for (int dx = 0; dx < 5; ++dx) {
            const int xx = min(max(x + dx - 2, 0), w - 1);
            v[dy * 5 + dx] = d[static_cast<long long>(yy) * Wp + xx];
        }
    }
    float m = median25(v);
    if (!(m > 0.f && m < max_disp)) m = 0.f;  // valid_mask = (d > 0) & (d < max_disp); setTo(0, ~valid)
    if (filtered) filtered[i] = m;
    // convertTo(CV_16UC1, 256.0): saturate_cast<ushort>(d * 256) = round half to even, clamp to [0, 65535]
    const float r = rintf(m * 256.0f);
    out[i] = static_cast<uint16_t>(fminf(fmaxf(r, 0.f), 65535.f));
}

}  // namespace

int launch_node_filter(const float* disp, uint16_t* out, float* filtered, int B, int Hp, int Wp, int top, int left,
                       int h, int w, float max_disp, hipStream_t s) {
    if (!disp || !out) return arg_error("node_filter: null pointer");
    if (B <= 0 || Hp <= 0 || Wp <= 0 || h <= 0 || w <= 0) return arg_error("node_filter: non-positive size");
    if (top < 0 || left < 0 || top + h > Hp || left + w > Wp) return arg_error("node_filter: window outside the map");
    const long long n = static_cast<long long>(B) * h * w;
    hipLaunchKernelGGL(node_filter_kernel, dim3(ceil_div(n, kThreads)), dim3(kThreads), 0, s, disp, out, filtered, Hp, Wp,
                       top, left, h, w, max_disp, n);
    return check_launch("node_filter");
}

int launch_preprocess(const uint8_t* img, float* out, int B, int H, int W, int Hp, int Wp, int top, int left,
                      int pad_normalized, hipStream_t s) {
    if (!img || !out) return arg_error("preprocess: null pointer");
    if (B <= 0 || H <= 0 || W <= 0 || Hp <= 0 || Wp <= 0) return arg_error("preprocess: non-positive size");
    if (top < 0 || left < 0 || top + H > Hp || left + W > Wp) return arg_error("preprocess: image does not fit the padded extent");
    const long long n = 3LL * B * Hp * Wp;
    hipLaunchKernelGGL(preprocess_kernel, dim3(ceil_div(n, kThreads)), dim3(kThreads), 0, s, img, out, H, W, Hp, Wp,
                       top, left, pad_normalized, n);
    return check_launch("preprocess");
}

int launch_disp_u16(const float* disp, uint16_t* out, int B, int Hp, int Wp, int top, int left, int h, int w,
                    hipStream_t s) {
    if (!disp || !out) return arg_error("disp_to_u16: null pointer");
    if (B <= 0 || Hp <= 0 || Wp <= 0 || h <= 0 || w <= 0) return arg_error("disp_to_u16: non-positive size");
    if (top < 0 || left < 0 || top + h > Hp || left + w > Wp) return arg_error("disp_to_u16: window outside the map");
    const long long n = static_cast<long long>(B) * h * w;
    hipLaunchKernelGGL(disp_u16_kernel, dim3(ceil_div(n, kThreads)), dim3(kThreads), 0, s, disp, out, Hp, Wp, top, left,
                       h, w, n);
    return check_launch("disp_to_u16");
}

}  // namespace esm

extern "C" {

int esm_preprocess_u8(const uint8_t* img, float* out, int B, int H, int W, int Hp, int Wp, int top, int left,
                      int pad_normalized, void* stream) {
    return esm::launch_preprocess(img, out, B, H, W, Hp, Wp, top, left, pad_normalized, esm::as_stream(stream));
}

int esm_node_filter_u16(const float* disp, uint16_t* out, float* filtered, int B, int Hp, int Wp, int top, int left,
                        int h, int w, float max_disp, void* stream) {
    return esm::launch_node_filter(disp, out, filtered, B, Hp, Wp, top, left, h, w, max_disp, esm::as_stream(stream));
}

int esm_disp_to_u16(const float* disp, uint16_t* out, int B, int Hp, int Wp, int top, int left, int h, int w,
                    void* stream) {
    return esm::launch_disp_u16(disp, out, B, Hp, Wp, top, left, h, w, esm::as_stream(stream));
}

}  // extern "C"
