// Native launch plan: the hot path (models/ESMStereo.py:700-745) recorded once as a list
// of kernel descriptors over caller-owned device buffers, launched eagerly or replayed as a
// single hipGraph (one host call per forward instead of ~70).  Optional hipEvent probe
// around one op measures that kernel's duration live on every run/replay.
#include <string>
#include <vector>

#include "common.h"

namespace esm {

int launch_gwc(const float*, const float*, const float*, float*, int, int, int, int, int, int, hipStream_t);
int launch_concat(const float*, const float*, float*, int, int, int, int, int, hipStream_t);
int launch_normcorr(const float*, const float*, float*, float*, int, int, int, int, int, hipStream_t);
int launch_regression(int, const float*, const float*, float*, int, int, int, int, hipStream_t);
int launch_conv(const esm_conv_desc*, hipStream_t);
int launch_smix(const esm_smix_desc*, hipStream_t);
int launch_fmnet(const esm_fmnet_desc*, hipStream_t);
int launch_shuffle_tail(const esm_shuffle_tail_desc*, hipStream_t);
int launch_shuffle_conv(const esm_shuffle_conv_desc*, hipStream_t);
namespace conv {
int launch_pair2(const esm_conv_desc&, const esm_conv_desc&, hipStream_t);
}
int launch_conf(const esm_conf_desc*, hipStream_t);

namespace {
thread_local std::string g_error;
}

void set_error(const std::string& msg) {
    g_error = msg;
    (void)hipGetLastError();  // never leave a sticky HIP error behind for the caller's runtime
}

}  // namespace esm

namespace {

enum OpKind { kConv = 1, kSmix = 2, kGwc = 3, kConcat = 4, kNormcorr = 5, kRegression = 6, kShuffleTail = 7, kFmnet = 9, kConf = 10, kShuffleConv = 12, kPair2 = 13 };

struct VolArgs {
    const float* L;
    const float* R;
    const float* att;
    float* V;
    float* work;
    int B, C, H, W, D, G;
};

struct RegArgs {
    int kind;
    const float* cost;
    float* out;
    int B, D, H, W;
};

struct Op {
    int kind = 0;
    esm_conv_desc conv{};
    esm_conv_desc conv2{};
    esm_smix_desc smix{};
    esm_fmnet_desc fm{};
    esm_shuffle_tail_desc st{};
    esm_shuffle_conv_desc sc{};
    VolArgs vol{};
    RegArgs reg{};
    esm_conf_desc cf{};
    int repeat = 1;  // launches per replay (esm_plan_set_repeat: 0 drops the op, 2 doubles it)
};

int run_op(const Op& op, hipStream_t s) {
    switch (op.kind) {
        case kConv: return esm::launch_conv(&op.conv, s);
        case kSmix: return esm::launch_smix(&op.smix, s);
        case kFmnet: return esm::launch_fmnet(&op.fm, s);
        case kShuffleTail: return esm::launch_shuffle_tail(&op.st, s);
        case kShuffleConv: return esm::launch_shuffle_conv(&op.sc, s);
        case kPair2: return esm::conv::launch_pair2(op.conv, op.conv2, s);
        case kConf: return esm::launch_conf(&op.cf, s);
        case kGwc:
            return esm::launch_gwc(op.vol.L, op.vol.R, op.vol.att, op.vol.V, op.vol.B, op.vol.C, op.vol.H, op.vol.W,
                                   op.vol.D, op.vol.G, s);
        case kConcat:
            return esm::launch_concat(op.vol.L, op.vol.R, op.vol.V, op.vol.B, op.vol.C, op.vol.H, op.vol.W, op.vol.D, s);
        case kNormcorr:
            return esm::launch_normcorr(op.vol.L, op.vol.R, op.vol.V, op.vol.work, op.vol.B, op.vol.C, op.vol.H,
                                        op.vol.W, op.vol.D, s);
        case kRegression:
            return esm::launch_regression(op.reg.kind, op.reg.cost, nullptr, op.reg.out, op.reg.B, op.reg.D, op.reg.H,
                                          op.reg.W, s);
        default: esm::set_error("plan: unknown op kind"); return ESM_ERR_ARG;
    }
}

// Nodes the next op captured on `s` will depend on (the last captured kernel node(s)).
std::vector<hipGraphNode_t> capture_frontier(hipStream_t s) {
    hipStreamCaptureStatus st;
    unsigned long long id = 0;
    hipGraph_t g = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t n = 0;
    if (hipStreamGetCaptureInfo_v2(s, &st, &id, &g, &deps, &n) != hipSuccess || !deps) return {};
    return std::vector<hipGraphNode_t>(deps, deps + n);
}

std::vector<hipGraphNode_t> successors(const std::vector<hipGraphNode_t>& nodes) {
    std::vector<hipGraphNode_t> out;
    for (auto nd : nodes) {
        size_t n = 0;
        if (hipGraphNodeGetDependentNodes(nd, nullptr, &n) != hipSuccess || n == 0) continue;
        std::vector<hipGraphNode_t> v(n);
        hipGraphNodeGetDependentNodes(nd, v.data(), &n);
        for (auto x : v) {
            bool seen = false;
            for (auto y : out) seen = seen || (x == y);
            if (!seen) out.push_back(x);
        }
    }
    return out;
}

std::vector<hipGraphNode_t> graph_roots(hipGraph_t g) {
    size_t n = 0;
    hipGraphGetRootNodes(g, nullptr, &n);
    std::vector<hipGraphNode_t> v(n);
    if (n) hipGraphGetRootNodes(g, v.data(), &n);
    return v;
}

}  // namespace

struct esm_plan {
    std::vector<Op> ops;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    hipStream_t cap_stream = nullptr;
    // probe
    int probe_index = -1;
    int ring = 0;
    std::vector<hipEvent_t> ev0, ev1;
    long long issued = 0, consumed = 0;
    hipGraphNode_t node0 = nullptr, node1 = nullptr;

    void clear_graph() {
        if (exec) hipGraphExecDestroy(exec);
        if (graph) hipGraphDestroy(graph);
        exec = nullptr;
        graph = nullptr;
        node0 = node1 = nullptr;
    }
    void clear_probe() {
        for (auto e : ev0) hipEventDestroy(e);
        for (auto e : ev1) hipEventDestroy(e);
        ev0.clear();
        ev1.clear();
        probe_index = -1;
        ring = 0;
        issued = consumed = 0;
    }
    ~esm_plan() {
        clear_graph();
        clear_probe();
        if (cap_stream) hipStreamDestroy(cap_stream);
    }
    // Launch every op on s; when `slot` >= 0 record the probe pair `slot` around the probed op.
    // Under stream capture the records become event-record graph nodes (hipEventRecordExternal).
    int launch_all(hipStream_t s, int slot, bool capture = false) {
        const unsigned flags = capture ? hipEventRecordExternal : 0u;
        for (int i = 0; i < static_cast<int>(ops.size()); ++i) {
            if (i == probe_index && slot >= 0) {
                const hipError_t e = hipEventRecordWithFlags(ev0[slot], s, flags);
                if (e != hipSuccess) {
                    esm::set_error(std::string("plan: hipEventRecord failed: ") + hipGetErrorString(e));
                    return ESM_ERR_RUNTIME;
                }
            }
            for (int r = 0; r < ops[i].repeat; ++r) {
                const int rc = run_op(ops[i], s);
                if (rc != ESM_OK) return rc;
            }
            if (i == probe_index && slot >= 0) {
                const hipError_t e = hipEventRecordWithFlags(ev1[slot], s, flags);
                if (e != hipSuccess) {
                    esm::set_error(std::string("plan: hipEventRecord failed: ") + hipGetErrorString(e));
                    return ESM_ERR_RUNTIME;
                }
            }
        }
        return ESM_OK;
    }
};

extern "C" {

const char* esm_last_error(void) { return esm::g_error.c_str(); }

int esm_version(void) { return 1; }

int esm_struct_size(int which) {
    switch (which) {
        case 0: return static_cast<int>(sizeof(esm_src));
        case 1: return static_cast<int>(sizeof(esm_conv_desc));
        case 2: return static_cast<int>(sizeof(esm_smix_stage));
        case 3: return static_cast<int>(sizeof(esm_smix_desc));
        case 4: return static_cast<int>(sizeof(esm_shuffle_tail_desc));
        case 5: return static_cast<int>(sizeof(esm_fmnet_desc));
        case 6: return static_cast<int>(sizeof(esm_conf_desc));
        case 8: return static_cast<int>(sizeof(esm_shuffle_conv_desc));
        default: return -1;
    }
}

esm_plan* esm_plan_create(void) { return new esm_plan(); }

void esm_plan_destroy(esm_plan* plan) { delete plan; }

static int add_op(esm_plan* plan, Op&& op) {
    if (!plan) return esm::arg_error("plan: null");
    plan->clear_graph();
    plan->ops.push_back(op);
    return static_cast<int>(plan->ops.size()) - 1;
}

int esm_plan_add_conv(esm_plan* plan, const esm_conv_desc* desc) {
    if (!desc) return esm::arg_error("plan: null conv desc");
    Op op;
    op.kind = kConv;
    op.conv = *desc;
    return add_op(plan, std::move(op));
}

int esm_plan_add_smix(esm_plan* plan, const esm_smix_desc* desc) {
    if (!desc) return esm::arg_error("plan: null smix desc");
    Op op;
    op.kind = kSmix;
    op.smix = *desc;
    return add_op(plan, std::move(op));
}

int esm_plan_add_fmnet(esm_plan* plan, const esm_fmnet_desc* desc) {
    if (!desc) return esm::arg_error("plan: null fmnet desc");
    Op op;
    op.kind = kFmnet;
    op.fm = *desc;
    return add_op(plan, std::move(op));
}

int esm_plan_add_shuffle_tail(esm_plan* plan, const esm_shuffle_tail_desc* desc) {
    if (!desc) return esm::arg_error("plan: null shuffle_tail desc");
    Op op;
    op.kind = kShuffleTail;
    op.st = *desc;
    return add_op(plan, std::move(op));
}

int esm_plan_add_conv_pair2(esm_plan* plan, const esm_conv_desc* a, const esm_conv_desc* b) {
    if (!a || !b) return esm::arg_error("plan: null conv pair desc");
    Op op;
    op.kind = kPair2;
    op.conv = *a;
    op.conv2 = *b;
    return add_op(plan, std::move(op));
}

int esm_plan_add_shuffle_conv(esm_plan* plan, const esm_shuffle_conv_desc* desc) {
    if (!desc) return esm::arg_error("plan: null shuffle_conv desc");
    Op op;
    op.kind = kShuffleConv;
    op.sc = *desc;
    return add_op(plan, std::move(op));
}

int esm_plan_add_gwc(esm_plan* plan, const float* L, const float* R, const float* att, float* V, int B, int C, int H,
                     int W, int D, int G) {
    Op op;
    op.kind = kGwc;
    op.vol = VolArgs{L, R, att, V, nullptr, B, C, H, W, D, G};
    return add_op(plan, std::move(op));
}

int esm_plan_add_concat(esm_plan* plan, const float* L, const float* R, float* V, int B, int C, int H, int W, int D) {
    Op op;
    op.kind = kConcat;
    op.vol = VolArgs{L, R, nullptr, V, nullptr, B, C, H, W, D, 0};
    return add_op(plan, std::move(op));
}

int esm_plan_add_normcorr(esm_plan* plan, const float* L, const float* R, float* V, float* work, int B, int C, int H,
                          int W, int D) {
    Op op;
    op.kind = kNormcorr;
    op.vol = VolArgs{L, R, nullptr, V, work, B, C, H, W, D, 0};
    return add_op(plan, std::move(op));
}

int esm_plan_add_regression(esm_plan* plan, int kind, const float* cost, float* out, int B, int D, int H, int W) {
    Op op;
    op.kind = kRegression;
    op.reg = RegArgs{kind, cost, out, B, D, H, W};
    return add_op(plan, std::move(op));
}

int esm_plan_add_conf(esm_plan* plan, const esm_conf_desc* desc) {
    if (!desc) return esm::arg_error("plan: null conf descriptor");
    Op op;
    op.kind = kConf;
    op.cf = *desc;
    return add_op(plan, std::move(op));
}

int esm_plan_num_ops(const esm_plan* plan) { return plan ? static_cast<int>(plan->ops.size()) : 0; }

int esm_plan_op_kind(const esm_plan* plan, int index) {
    if (!plan || index < 0 || index >= static_cast<int>(plan->ops.size())) return 0;
    return plan->ops[index].kind;
}

static int next_slot(esm_plan* plan) {
    if (plan->probe_index < 0) return -1;
    const int slot = static_cast<int>(plan->issued % plan->ring);
    plan->issued++;
    if (plan->issued - plan->consumed > plan->ring) plan->consumed = plan->issued - plan->ring;
    return slot;
}

int esm_plan_set_conv_hint(esm_plan* plan, int index, int hint) {
    if (!plan) return esm::arg_error("plan: null");
    if (index < 0 || index >= static_cast<int>(plan->ops.size()) || plan->ops[index].kind != kConv)
        return esm::arg_error("plan: op is not a conv");
    const int prev = plan->ops[index].conv.hint;
    plan->clear_graph();
    // the tile-order bit (30) is the host's per-launch choice, not a form: kept across tuning hints
    plan->ops[index].conv.hint = (hint & ~esm::kHintXcd) | (prev & esm::kHintXcd);
    return prev & ~esm::kHintXcd;
}

int esm_plan_set_repeat(esm_plan* plan, int index, int repeat) {
    if (!plan) return esm::arg_error("plan: null");
    if (index < 0 || index >= static_cast<int>(plan->ops.size())) return esm::arg_error("plan: op index out of range");
    if (repeat < 0 || repeat > 8) return esm::arg_error("plan: repeat must be 0..8");
    if (repeat == 0 && index == plan->probe_index) return esm::arg_error("plan: cannot drop the probed op");
    plan->clear_graph();
    const int prev = plan->ops[index].repeat;
    plan->ops[index].repeat = repeat;
    return prev;
}

int esm_plan_run(esm_plan* plan, void* stream) {
    if (!plan) return esm::arg_error("plan: null");
    return plan->launch_all(esm::as_stream(stream), next_slot(plan));
}

int esm_plan_run_op(esm_plan* plan, int index, int reps, void* stream) {
    if (!plan) return esm::arg_error("plan: null");
    if (index < 0 || index >= static_cast<int>(plan->ops.size())) return esm::arg_error("plan: op index out of range");
    if (reps < 1) return esm::arg_error("plan: reps must be >= 1");
    const hipStream_t s = esm::as_stream(stream);
    for (int r = 0; r < reps; ++r) {
        const int rc = run_op(plan->ops[index], s);
        if (rc != ESM_OK) return rc;
    }
    return ESM_OK;
}

int esm_plan_graph_build(esm_plan* plan, void* stream) {
    if (!plan) return esm::arg_error("plan: null");
    (void)stream;
    plan->clear_graph();
    if (!plan->cap_stream && hipStreamCreateWithFlags(&plan->cap_stream, hipStreamNonBlocking) != hipSuccess) {
        esm::set_error("plan: cannot create capture stream");
        return ESM_ERR_RUNTIME;
    }
    if (hipStreamBeginCapture(plan->cap_stream, hipStreamCaptureModeThreadLocal) != hipSuccess) {
        esm::set_error("plan: hipStreamBeginCapture failed");
        return ESM_ERR_RUNTIME;
    }
    // Capture the launch list; around the probed op remember the capture frontier so the
    // event-record nodes can be spliced in after capture (records inside capture are refused).
    std::vector<hipGraphNode_t> before, after;
    int rc = ESM_OK;
    for (int i = 0; i < static_cast<int>(plan->ops.size()) && rc == ESM_OK; ++i) {
        if (i == plan->probe_index) before = capture_frontier(plan->cap_stream);
        for (int r = 0; r < plan->ops[i].repeat && rc == ESM_OK; ++r) rc = run_op(plan->ops[i], plan->cap_stream);
        if (i == plan->probe_index) after = capture_frontier(plan->cap_stream);
    }
    hipGraph_t g = nullptr;
    const hipError_t ec = hipStreamEndCapture(plan->cap_stream, &g);
    if (rc != ESM_OK) {
        if (g) hipGraphDestroy(g);
        return rc;
    }
    if (ec != hipSuccess || !g) {
        esm::set_error(std::string("plan: hipStreamEndCapture failed: ") + hipGetErrorString(ec));
        return ESM_ERR_RUNTIME;
    }
    plan->graph = g;
    if (plan->probe_index >= 0) {
        if (after.empty()) {
            plan->clear_graph();
            esm::set_error("plan: could not locate the probed op in the captured graph");
            return ESM_ERR_UNSUPPORTED;
        }
        const std::vector<hipGraphNode_t> first = before.empty() ? graph_roots(g) : successors(before);
        const std::vector<hipGraphNode_t> next = successors(after);
        hipError_t e = hipGraphAddEventRecordNode(&plan->node0, g, before.data(), before.size(), plan->ev0[0]);
        for (size_t k = 0; e == hipSuccess && k < first.size(); ++k) e = hipGraphAddDependencies(g, &plan->node0, &first[k], 1);
        if (e == hipSuccess) e = hipGraphAddEventRecordNode(&plan->node1, g, after.data(), after.size(), plan->ev1[0]);
        for (size_t k = 0; e == hipSuccess && k < next.size(); ++k) e = hipGraphAddDependencies(g, &plan->node1, &next[k], 1);
        if (e != hipSuccess) {
            plan->clear_graph();
            esm::set_error(std::string("plan: cannot add probe event nodes: ") + hipGetErrorString(e));
            return ESM_ERR_UNSUPPORTED;
        }
    }
    const hipError_t ei = hipGraphInstantiate(&plan->exec, g, nullptr, nullptr, 0);
    if (ei != hipSuccess) {
        plan->clear_graph();
        esm::set_error(std::string("plan: hipGraphInstantiate failed: ") + hipGetErrorString(ei));
        return ESM_ERR_RUNTIME;
    }
    return ESM_OK;
}

int esm_plan_graph_launch(esm_plan* plan, void* stream) {
    if (!plan || !plan->exec) return esm::arg_error("plan: graph not built");
    const int slot = next_slot(plan);
    if (slot >= 0) {
        if (hipGraphExecEventRecordNodeSetEvent(plan->exec, plan->node0, plan->ev0[slot]) != hipSuccess ||
            hipGraphExecEventRecordNodeSetEvent(plan->exec, plan->node1, plan->ev1[slot]) != hipSuccess) {
            esm::set_error("plan: cannot retarget probe events");
            return ESM_ERR_RUNTIME;
        }
    }
    const hipError_t e = hipGraphLaunch(plan->exec, esm::as_stream(stream));
    if (e != hipSuccess) {
        esm::set_error(std::string("plan: hipGraphLaunch failed: ") + hipGetErrorString(e));
        return ESM_ERR_LAUNCH;
    }
    return ESM_OK;
}

int esm_plan_set_probe(esm_plan* plan, int index, int ring) {
    if (!plan) return esm::arg_error("plan: null");
    plan->clear_graph();
    plan->clear_probe();
    if (index < 0) return ESM_OK;
    if (index >= static_cast<int>(plan->ops.size()) || ring <= 0 || ring > 4096)
        return esm::arg_error("plan: bad probe index/ring");
    plan->ev0.resize(ring);
    plan->ev1.resize(ring);
    for (int i = 0; i < ring; ++i) {
        if (hipEventCreate(&plan->ev0[i]) != hipSuccess || hipEventCreate(&plan->ev1[i]) != hipSuccess) {
            esm::set_error("plan: hipEventCreate failed");
            return ESM_ERR_RUNTIME;
        }
    }
    plan->probe_index = index;
    plan->ring = ring;
    return ESM_OK;
}

int esm_plan_probe_read(esm_plan* plan, float* ms, int max) {
    if (!plan || !ms) return esm::arg_error("plan: null");
    int n = 0;
    while (plan->consumed < plan->issued && n < max) {
        const int slot = static_cast<int>(plan->consumed % plan->ring);
        float t = 0.f;
        if (hipEventElapsedTime(&t, plan->ev0[slot], plan->ev1[slot]) != hipSuccess) {
            esm::set_error("plan: hipEventElapsedTime failed (synchronise first)");
            return ESM_ERR_RUNTIME;
        }
        ms[n++] = t;
        plan->consumed++;
    }
    return n;
}

}  // extern "C"
