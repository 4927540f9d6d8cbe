// Host-side AddressSanitizer / LeakSanitizer check of the C ABI (include/esmstereo_amd.h).
//
// Built by scripts/asan_host.sh against objects compiled with the host half instrumented
// (device code is untouched) and run on a machine WITHOUT a GPU: every entry point's descriptor
// validation, error reporting and the plan container are driven with valid, invalid and randomly
// mutated arguments.  Descriptors that pass validation reach the launch, which fails with "no
// device"; the device pointers below are host dummies and are never dereferenced by host code.
// Refuses to run when a GPU is visible (a mutated descriptor would then really launch).
//
// Checks: no ASan report (heap/stack/global overflow, use-after-free, leaks at exit), every
// return code is ESM_OK or one of the ESM_ERR_* codes, and every failure leaves a message in
// esm_last_error().
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "esmstereo_amd.h"

namespace {

int g_checked = 0, g_fail = 0;
std::mt19937_64 rng(20261017);

float g_dummy[64];
float* P = g_dummy;  // a non-null "device" pointer the host never reads through

void check(int rc, const char* what) {
    ++g_checked;
    const bool known = rc == ESM_OK || rc == ESM_ERR_ARG || rc == ESM_ERR_LAUNCH || rc == ESM_ERR_UNSUPPORTED ||
                       rc == ESM_ERR_RUNTIME;
    if (!known) {
        std::fprintf(stderr, "FAIL %s: unknown return code %d\n", what, rc);
        ++g_fail;
        return;
    }
    if (rc < 0 && (!esm_last_error() || !esm_last_error()[0])) {
        std::fprintf(stderr, "FAIL %s: rc %d without a message\n", what, rc);
        ++g_fail;
    }
}

void expect_err(int rc, const char* what) {
    check(rc, what);
    if (rc >= 0) {
        std::fprintf(stderr, "FAIL %s: expected an error, got %d\n", what, rc);
        ++g_fail;
    }
}

int pick_int() {
    static const int v[] = {-7, -1, 0, 1, 2, 3, 4, 5, 7, 8, 12, 16, 24, 31, 32, 33, 48, 64, 65, 96, 1 << 20, 0x7fffffff};
    return v[rng() % (sizeof(v) / sizeof(v[0]))];
}

// Mutate n random 32-bit words of a POD descriptor: sizes, strides, flags and pointers alike.
// Pointer words are only ever replaced by 0 or P (a wild pointer would be a false positive: the
// host never reads through them, but a null is a legitimate invalid argument).
template <class T>
T mutate(const T& base, int n, const std::vector<size_t>& ptr_offsets) {
    T d = base;
    auto* w = reinterpret_cast<unsigned char*>(&d);
    for (int i = 0; i < n; ++i) {
        const size_t words = sizeof(T) / 4;
        const size_t k = rng() % words;
        bool is_ptr = false;
        for (size_t off : ptr_offsets)
            if (k * 4 >= off && k * 4 < off + sizeof(void*)) {
                is_ptr = true;
                const void* v = (rng() & 1) ? nullptr : static_cast<const void*>(P);
                std::memcpy(w + off, &v, sizeof(void*));
            }
        if (!is_ptr) {
            const int v = pick_int();
            std::memcpy(w + 4 * k, &v, 4);
        }
    }
    return d;
}

esm_src src(int C, long long sb, long long sc, long long sd, long long sh) {
    esm_src s{};
    s.ptr = P;
    s.C = C;
    s.sb = sb;
    s.sc = sc;
    s.sd = sd;
    s.sh = sh;
    return s;
}

// A valid 3x3x3 s1 p1 3-D BasicConv 8 -> 8 on 4 x 6 x 20 (batch 1).
esm_conv_desc conv3d_base() {
    esm_conv_desc d{};
    const int D = 4, H = 6, W = 20;
    d.src[0] = src(8, 8LL * D * H * W, D * H * W, H * W, W);
    d.nsrc = 1;
    d.B = 1;
    d.Cin = 8;
    d.Di = d.Do = D;
    d.Hi = d.Ho = H;
    d.Wi = d.Wo = W;
    d.kd = d.kh = d.kw = 3;
    d.stride = 1;
    d.pd = d.ph = d.pw = 1;
    d.Cout = 8;
    d.cin_pad = 16;
    d.cout_pad = 32;
    d.w = P;
    d.scale = P;
    d.shift = P;
    d.act = ESM_ACT_GELU;
    d.shuffle = 1;
    d.out = P;
    d.ob = 8LL * D * H * W;
    d.oc = D * H * W;
    d.od = H * W;
    d.oh = W;
    d.post_scale = 1.f;
    d.post_scale2 = 1.f;
    return d;
}

// A valid 3x3 s1 p1 2-D conv 16 -> 16 on 24 x 78.
esm_conv_desc conv2d_base() {
    esm_conv_desc d = conv3d_base();
    const int H = 24, W = 78;
    d.src[0] = src(16, 16LL * H * W, H * W, 0, W);
    d.Cin = 16;
    d.Di = d.Do = 1;
    d.Hi = d.Ho = H;
    d.Wi = d.Wo = W;
    d.kd = 1;
    d.pd = 0;
    d.Cout = 16;
    d.ob = 16LL * H * W;
    d.oc = H * W;
    d.od = 0;
    d.oh = W;
    return d;
}

std::vector<size_t> conv_ptrs() {
    std::vector<size_t> v;
    for (int i = 0; i < ESM_MAX_SRC; ++i) v.push_back(offsetof(esm_conv_desc, src) + i * sizeof(esm_src));
    for (size_t o : {offsetof(esm_conv_desc, w), offsetof(esm_conv_desc, scale), offsetof(esm_conv_desc, shift),
                     offsetof(esm_conv_desc, mul), offsetof(esm_conv_desc, res), offsetof(esm_conv_desc, out),
                     offsetof(esm_conv_desc, up), offsetof(esm_conv_desc, out2)})
        v.push_back(o);
    return v;
}

esm_smix_stage stage() { return esm_smix_stage{P, P, P, P, P}; }

esm_fmnet_desc fmnet_base() {
    esm_fmnet_desc d{};
    d.x = P;
    d.out = P + 1;
    d.dw_w[0] = d.dw_w[1] = P;
    d.dw_b[0] = d.dw_b[1] = P;
    d.dw_k = 7;
    for (auto& s : d.stage) s = stage();
    d.B = 1;
    d.C = 8;
    d.H = 24;
    d.W = 78;
    d.conv0_w = d.conv0_b = d.conv2_w = d.conv2_b = P;
    d.hid = 24;
    return d;
}

esm_smix_desc smix_base() {
    esm_smix_desc d{};
    d.x = P;
    d.out = P + 1;
    d.dw_w = P;
    d.dw_b = P;
    d.dw_k = 7;
    d.nstages = 2;
    d.stage[0] = d.stage[1] = stage();
    d.B = 1;
    d.C = 16;
    d.H = 24;
    d.W = 78;
    return d;
}

esm_shuffle_tail_desc tail_base() {
    esm_shuffle_tail_desc d{};
    d.x = P;
    d.xb = 8 * 24 * 78;
    d.xc = 24 * 78;
    d.xh = 78;
    d.up_w = d.up_b = d.tail_w = d.tail_b = P;
    d.out = P;
    d.ob = 96 * 312;
    d.oh = 312;
    d.B = 1;
    d.nf = 8;
    d.H = 24;
    d.W = 78;
    d.r = 4;
    return d;
}

esm_shuffle_conv_desc sconv_base() {
    esm_shuffle_conv_desc d{};
    d.st = tail_base();
    d.st.r = 2;
    d.st.ob = 48 * 156;
    d.st.oh = 156;
    d.w = d.scale = d.shift = P;
    d.out = P;
    d.C = 16;
    d.ob = 16 * 24 * 78;
    d.oc = 24 * 78;
    d.oh = 78;
    d.cin_pad = 16;
    d.cout_pad = 32;
    return d;
}

// the S 4x stage: spx_4x[1] computed inside the row-form launch (pre_x; st.x NULL)
esm_shuffle_conv_desc sconv_pre_base() {
    esm_shuffle_conv_desc d = sconv_base();
    d.st.x = nullptr;
    d.st.r = 4;
    d.st.H = 96;
    d.st.W = 312;
    d.st.xb = 8 * 96 * 312;
    d.st.xc = 96 * 312;
    d.st.xh = 312;
    d.st.ob = 384 * 1248;
    d.st.oh = 1248;
    d.ob = 16 * 192 * 624;
    d.oc = 192 * 624;
    d.oh = 624;
    d.pre_x = d.pre_w = d.pre_scale = d.pre_shift = P;
    d.pb = 16 * 96 * 312;
    d.pc = 96 * 312;
    d.ph = 312;
    d.pre_cin = 16;
    d.pre_cin_pad = 16;
    d.pre_cout_pad = 32;
    return d;
}

void fuzz_conv(int iters) {
    const auto ptrs = conv_ptrs();
    for (const esm_conv_desc& base : {conv3d_base(), conv2d_base()}) {
        check(esm_conv_f32(&base, nullptr), "conv base");
        for (int i = 0; i < iters; ++i) {
            esm_conv_desc d = mutate(base, 1 + static_cast<int>(rng() % 3), ptrs);
            if (rng() % 4 == 0) d.hint = static_cast<int>(rng() & 0x3fffffff);
            if (rng() % 8 == 0) d.transposed = 1;
            check(esm_conv_f32(&d, nullptr), "conv fuzz");
            esm_conv_desc b = mutate(conv2d_base(), static_cast<int>(rng() % 2), ptrs);
            check(esm_conv_pair2_f32(&d, &b, nullptr), "pair2 fuzz");
        }
    }
    expect_err(esm_conv_f32(nullptr, nullptr), "conv null");
    expect_err(esm_conv_pair2_f32(nullptr, nullptr, nullptr), "pair2 null");
}

template <class T>
void fuzz_desc(const T& base, int (*fn)(const T*, void*), const std::vector<size_t>& ptrs, const char* name,
               int iters) {
    check(fn(&base, nullptr), name);
    for (int i = 0; i < iters; ++i) {
        const T d = mutate(base, 1 + static_cast<int>(rng() % 3), ptrs);
        check(fn(&d, nullptr), name);
    }
    expect_err(fn(nullptr, nullptr), name);
}

void fuzz_flat(int iters) {
    for (int i = 0; i < iters; ++i) {
        const int B = pick_int(), C = pick_int(), H = pick_int(), W = pick_int(), D = pick_int(), G = pick_int();
        const float* a = (rng() % 8) ? P : nullptr;
        check(esm_gwc_volume_f32(a, P, (rng() & 1) ? P : nullptr, P, B, C, H, W, D, G, nullptr), "gwc");
        check(esm_concat_volume_f32(a, P, P, B, C, H, W, D, nullptr), "concat");
        check(esm_normcorr_volume_f32(a, P, P, nullptr, B, C, H, W, D, nullptr), "normcorr");
        check(esm_disp_regression_f32(a, P, B, D, H, W, nullptr), "dispreg");
        check(esm_topk2_regression_f32(a, (rng() & 1) ? P : nullptr, P, B, D, H, W, nullptr), "topk2");
        check(esm_topk_regression_f32(a, (rng() & 1) ? P : nullptr, P, B, D, H, W, pick_int(), nullptr), "topk");
        const uint8_t img[4] = {};
        uint16_t o16[4];
        check(esm_preprocess_u8((rng() % 8) ? img : nullptr, P, B, H, W, pick_int(), pick_int(), pick_int(), pick_int(),
                                static_cast<int>(rng() % 3), nullptr),
              "preprocess");
        check(esm_disp_to_u16(a, o16, B, H, W, pick_int(), pick_int(), pick_int(), pick_int(), nullptr), "to_u16");
        check(esm_node_filter_u16(a, o16, (rng() & 1) ? P : nullptr, B, H, W, pick_int(), pick_int(), pick_int(),
                                  pick_int(), 192.f, nullptr),
              "node_filter");
        esm_conf_desc cf{};
        cf.op = static_cast<int>(rng() % 7);
        cf.B = B;
        cf.C = C;
        cf.D = D;
        cf.H = H;
        cf.W = W;
        for (auto& x : cf.x) x = (rng() % 6) ? P : nullptr;
        cf.out = (rng() % 8) ? P : nullptr;
        check(esm_conf_f32(&cf, nullptr), "conf");
    }
    expect_err(esm_conf_f32(nullptr, nullptr), "conf null");
}

void plans(int iters) {
    for (int it = 0; it < iters; ++it) {
        esm_plan* p = esm_plan_create();
        const int n = 1 + static_cast<int>(rng() % 80);
        for (int i = 0; i < n; ++i) {
            const esm_conv_desc c = conv3d_base(), c2 = conv2d_base();
            const esm_fmnet_desc f = fmnet_base();
            const esm_smix_desc s = smix_base();
            const esm_shuffle_tail_desc t = tail_base();
            const esm_shuffle_conv_desc sc = sconv_base();
            esm_conf_desc cf{};
            cf.op = ESM_CONF_SIGMOID;
            cf.B = cf.C = cf.H = cf.W = 1;
            cf.x[0] = P;
            cf.out = P;
            int rc = 0;
            switch (rng() % 12) {
                case 0: rc = esm_plan_add_conv(p, &c); break;
                case 1: rc = esm_plan_add_conv_pair2(p, &c2, &c2); break;
                case 2: rc = esm_plan_add_fmnet(p, &f); break;
                case 3: rc = esm_plan_add_smix(p, &s); break;
                case 4: rc = esm_plan_add_shuffle_tail(p, &t); break;
                case 5: rc = esm_plan_add_shuffle_conv(p, &sc); break;
                case 6: rc = esm_plan_add_gwc(p, P, P, nullptr, P, 1, 64, 24, 78, 48, 32); break;
                case 7: rc = esm_plan_add_concat(p, P, P, P, 1, 16, 24, 78, 48); break;
                case 8: rc = esm_plan_add_normcorr(p, P, P, P, nullptr, 1, 64, 24, 78, 48); break;
                case 9: rc = esm_plan_add_regression(p, static_cast<int>(rng() % 6), P, P, 1, 48, 24, 78); break;
                case 10: rc = esm_plan_add_conf(p, &cf); break;
                default: rc = esm_plan_add_conv(p, nullptr); break;
            }
            check(rc >= 0 ? ESM_OK : rc, "plan add");
        }
        const int nops = esm_plan_num_ops(p);
        for (int k = 0; k < 8; ++k) {
            const int idx = static_cast<int>(rng() % (nops + 4)) - 2;
            check(esm_plan_op_kind(p, idx) >= 0 ? 0 : esm_plan_op_kind(p, idx), "op_kind");
            check(esm_plan_set_conv_hint(p, idx, pick_int()) >= 0 ? 0 : ESM_ERR_ARG, "set_hint");
            check(esm_plan_set_repeat(p, idx, pick_int()) >= 0 ? 0 : ESM_ERR_ARG, "set_repeat");
        }
        check(esm_plan_run_op(p, static_cast<int>(rng() % (nops + 2)) - 1, pick_int(), nullptr), "run_op");
        {  // zero-copy rebinding: random ranges around the dummy pointer, moved to other dummies and back
            const int nb = static_cast<int>(rng() % 4);
            const void* olds[3];
            const void* news[3];
            uint64_t bytes[3];
            for (int k = 0; k < 3; ++k) {
                olds[k] = g_dummy + (rng() % 8);
                news[k] = g_dummy + (rng() % 8);
                bytes[k] = (rng() % 3 == 0) ? 0 : 4 * (1 + rng() % 64);
            }
            const int rc = esm_plan_rebind(p, nb, nb ? olds : nullptr, nb ? bytes : nullptr, nb ? news : nullptr);
            check(rc >= 0 ? 0 : rc, "rebind");
            check(esm_plan_rebind(p, nb, nb ? news : nullptr, nb ? bytes : nullptr, nb ? olds : nullptr) >= 0 ? 0 : ESM_ERR_ARG,
                  "rebind back");
        }
        expect_err(esm_plan_rebind(p, 1, nullptr, nullptr, nullptr), "rebind null arrays");
        if (it % 16 == 0) {
            // no device here: these reach the runtime and must fail cleanly (stream / graph / events)
            check(esm_plan_run(p, nullptr), "plan run");
            check(esm_plan_graph_build(p, nullptr), "graph build");
            check(esm_plan_graph_launch(p, nullptr), "graph launch");
            check(esm_plan_set_probe(p, static_cast<int>(rng() % (nops + 1)), pick_int()), "set_probe");
            float ms[8];
            check(esm_plan_probe_read(p, ms, 8) >= 0 ? 0 : ESM_ERR_ARG, "probe_read");
        }
        esm_plan_destroy(p);
    }
    if (esm_plan_num_ops(nullptr) != 0) {
        std::fprintf(stderr, "FAIL num_ops(null) != 0\n");
        ++g_fail;
    }
    expect_err(esm_plan_run(nullptr, nullptr), "run null");
    expect_err(esm_plan_graph_launch(nullptr, nullptr), "graph launch null");
    esm_plan_destroy(nullptr);
}

}  // namespace

int main(int argc, char** argv) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0) {
        std::fprintf(stderr, "abi_check: a GPU is visible; this check drives launches with dummy pointers and only "
                             "runs without one\n");
        return 2;
    }
    const int iters = argc > 1 ? std::atoi(argv[1]) : 4000;
    check(esm_version() > 0 ? 0 : ESM_ERR_ARG, "version");
    for (int i = -2; i < 12; ++i) (void)esm_struct_size(i);
    fuzz_conv(iters);
    const std::vector<size_t> fm_ptrs = {offsetof(esm_fmnet_desc, x), offsetof(esm_fmnet_desc, out),
                                         offsetof(esm_fmnet_desc, dw_w), offsetof(esm_fmnet_desc, dw_w) + 8,
                                         offsetof(esm_fmnet_desc, dw_b), offsetof(esm_fmnet_desc, dw_b) + 8,
                                         offsetof(esm_fmnet_desc, conv0_w), offsetof(esm_fmnet_desc, conv0_b),
                                         offsetof(esm_fmnet_desc, conv2_w), offsetof(esm_fmnet_desc, conv2_b),
                                         offsetof(esm_fmnet_desc, work)};
    std::vector<size_t> fm_all = fm_ptrs;
    for (int s = 0; s < 4; ++s)
        for (int j = 0; j < 5; ++j) fm_all.push_back(offsetof(esm_fmnet_desc, stage) + s * sizeof(esm_smix_stage) + 8 * j);
    fuzz_desc<esm_fmnet_desc>(fmnet_base(), esm_fmnet_f32, fm_all, "fmnet", iters);
    std::vector<size_t> sm_ptrs = {offsetof(esm_smix_desc, x), offsetof(esm_smix_desc, out), offsetof(esm_smix_desc, res),
                                   offsetof(esm_smix_desc, dw_w), offsetof(esm_smix_desc, dw_b)};
    for (int s = 0; s < ESM_SMIX_MAX_STAGES; ++s)
        for (int j = 0; j < 5; ++j) sm_ptrs.push_back(offsetof(esm_smix_desc, stage) + s * sizeof(esm_smix_stage) + 8 * j);
    fuzz_desc<esm_smix_desc>(smix_base(), esm_smix_f32, sm_ptrs, "smix", iters);
    const std::vector<size_t> st_ptrs = {offsetof(esm_shuffle_tail_desc, x),      offsetof(esm_shuffle_tail_desc, up_w),
                                         offsetof(esm_shuffle_tail_desc, up_b),   offsetof(esm_shuffle_tail_desc, tail_w),
                                         offsetof(esm_shuffle_tail_desc, tail_b), offsetof(esm_shuffle_tail_desc, out)};
    fuzz_desc<esm_shuffle_tail_desc>(tail_base(), esm_shuffle_tail_f32, st_ptrs, "shuffle_tail", iters);
    std::vector<size_t> sc_ptrs = st_ptrs;
    for (size_t o : {offsetof(esm_shuffle_conv_desc, w), offsetof(esm_shuffle_conv_desc, scale),
                     offsetof(esm_shuffle_conv_desc, shift), offsetof(esm_shuffle_conv_desc, out)})
        sc_ptrs.push_back(o);
    fuzz_desc<esm_shuffle_conv_desc>(sconv_base(), esm_shuffle_conv_f32, sc_ptrs, "shuffle_conv", iters);
    for (size_t o : {offsetof(esm_shuffle_conv_desc, pre_x), offsetof(esm_shuffle_conv_desc, pre_w),
                     offsetof(esm_shuffle_conv_desc, pre_scale), offsetof(esm_shuffle_conv_desc, pre_shift)})
        sc_ptrs.push_back(o);
    fuzz_desc<esm_shuffle_conv_desc>(sconv_pre_base(), esm_shuffle_conv_f32, sc_ptrs, "shuffle_conv pre", iters);
    fuzz_flat(iters);
    plans(iters / 20 + 1);
    std::printf("abi_check: %d calls checked, %d failures\n", g_checked, g_fail);
    return g_fail ? 1 : 0;
}
