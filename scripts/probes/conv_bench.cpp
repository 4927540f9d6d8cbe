// Native timing harness for single library launches (no Python in the loop): the ref4x.agg_1 pair
// and its two layers at S-K size (192x624) in every form, back to back between one hipEvent pair.
//   hipcc -O3 --offload-arch=gfx950 -o scripts/probes/conv_bench scripts/probes/conv_bench.cpp \
//       -Lesmstereo_amd -lesmstereo_amd -Wl,-rpath,'$ORIGIN/../../esmstereo_amd'
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/esmstereo_amd.h"

static float* dalloc(size_t n, float v) {
    float* p = nullptr;
    (void)hipMalloc(&p, n * 4);
    std::vector<float> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = v * static_cast<float>((i * 2654435761u) % 1000) / 1000.f - 0.5f * v;
    (void)hipMemcpy(p, h.data(), n * 4, hipMemcpyHostToDevice);
    return p;
}

static esm_conv_desc conv2d(const float* const* srcs, const int* cs, int nsrc, int H, int W, int Cout, int k,
                            const float* w, const float* scale, const float* shift, float* out, int hint) {
    esm_conv_desc d;
    std::memset(&d, 0, sizeof d);
    int cin = 0;
    for (int i = 0; i < nsrc; ++i) {
        d.src[i].ptr = srcs[i];
        d.src[i].C = cs[i];
        d.src[i].sb = static_cast<long long>(cs[i]) * H * W;
        d.src[i].sc = static_cast<long long>(H) * W;
        d.src[i].sh = W;
        cin += cs[i];
    }
    d.nsrc = nsrc;
    d.B = 1;
    d.Cin = cin;
    d.Di = d.Do = 1;
    d.Hi = d.Ho = H;
    d.Wi = d.Wo = W;
    d.kd = 1;
    d.kh = d.kw = k;
    d.stride = 1;
    d.ph = d.pw = k / 2;
    d.Cout = Cout;
    d.cin_pad = (cin + 15) / 16 * 16;
    d.cout_pad = (Cout + 31) / 32 * 32;
    d.w = w;
    d.scale = scale;
    d.shift = shift;
    d.act = ESM_ACT_GELU;
    d.shuffle = 1;
    d.out = out;
    d.ob = static_cast<long long>(Cout) * H * W;
    d.oc = static_cast<long long>(H) * W;
    d.oh = W;
    d.post_scale = d.post_scale2 = 1.f;
    d.hint = hint;
    return d;
}

template <typename F>
static float timeit(F f, int reps = 100) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    if (f() < 0) {
        printf("  launch failed: %s\n", esm_last_error());
        return -1.f;
    }
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, nullptr);
    for (int i = 0; i < reps; ++i) f();
    (void)hipEventRecord(b, nullptr);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / reps * 1e3f;
}

int main() {
    const int H = 192, W = 624;
    const int cs[3] = {16, 16, 24};
    // the three sources carved out of one allocation (as the plan's arena does)
    float* pool = dalloc(56ull * H * W + 4096, 2.f);
    const float* srcs[3] = {pool + 1024, pool + 1024 + 16ull * H * W, pool + 1024 + 32ull * H * W};
    const float* one[1] = {pool + 1024};
    const int c56[1] = {56};
    float* wa = dalloc(64 * 32, 0.3f);
    float* wb = dalloc(9 * 16 * 32, 0.3f);
    float* sc = dalloc(32, 0.2f);
    float* sh = dalloc(32, 0.2f);
    float* mid = dalloc(16ull * H * W, 0.f);
    float* out = dalloc(16ull * H * W, 0.f);
    const float* mids[1] = {mid};
    const int c16[1] = {16};
    printf("ref4x.agg_1 at %dx%d (us per launch, back to back)\n", H, W);
    const int hints[] = {0, 1 << 21, 1 << 22};
    for (int h : hints) {
        esm_conv_desc a = conv2d(srcs, cs, 3, H, W, 16, 1, wa, sc, sh, mid, h);
        esm_conv_desc b = conv2d(mids, c16, 1, H, W, 16, 3, wb, sc, sh, out, h);
        const float ta = timeit([&] { return esm_conv_f32(&a, nullptr); });
        const float tb = timeit([&] { return esm_conv_f32(&b, nullptr); });
        esm_conv_desc a1 = conv2d(one, c56, 1, H, W, 16, 1, wa, sc, sh, mid, h);
        const float t1 = timeit([&] { return esm_conv_f32(&a1, nullptr); });
        printf("hint %#8x: 1x1 56->16 (3 sources) %7.2f  (1 source) %7.2f | 3x3 16->16 %7.2f\n", h, ta, t1, tb);
    }
    for (int legacy = 0; legacy < 2; ++legacy) {
        esm_conv_desc a = conv2d(srcs, cs, 3, H, W, 16, 1, wa, sc, sh, nullptr, legacy ? (1 << 23) : 0);
        esm_conv_desc b = conv2d(srcs, cs, 0, H, W, 16, 3, wb, sc, sh, out, 0);
        b.Cin = 16;
        b.cin_pad = 16;
        const float t = timeit([&] { return esm_conv_pair_f32(&a, &b, nullptr); });
        printf("pair (%s): %7.2f\n", legacy ? "LDS-weight kernel" : "lean", t);
    }
    return 0;
}
