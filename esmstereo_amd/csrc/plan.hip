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

namespace {
thread_local std::string g_error;
}

void set_error(const std::string& msg) { g_error = msg; }

}  // namespace esm

namespace {

enum OpKind { kConv = 1, kSmix = 2, kGwc = 3, kConcat = 4, kNormcorr = 5, kRegression = 6 };

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
    esm_smix_desc smix{};
    VolArgs vol{};
    RegArgs reg{};
};

int run_op(const Op& op, hipStream_t s) {
    switch (op.kind) {
        case kConv: return esm::launch_conv(&op.conv, s);
        case kSmix: return esm::launch_smix(&op.smix, s);
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
    int launch_all(hipStream_t s, int slot) {
        for (int i = 0; i < static_cast<int>(ops.size()); ++i) {
            if (i == probe_index && slot >= 0 && hipEventRecord(ev0[slot], s) != hipSuccess) {
                esm::set_error("plan: hipEventRecord failed");
                return ESM_ERR_RUNTIME;
            }
            const int rc = run_op(ops[i], s);
            if (rc != ESM_OK) return rc;
            if (i == probe_index && slot >= 0 && hipEventRecord(ev1[slot], s) != hipSuccess) {
                esm::set_error("plan: hipEventRecord failed");
                return ESM_ERR_RUNTIME;
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

int esm_plan_run(esm_plan* plan, void* stream) {
    if (!plan) return esm::arg_error("plan: null");
    return plan->launch_all(esm::as_stream(stream), next_slot(plan));
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
    const int rc = plan->launch_all(plan->cap_stream, plan->probe_index >= 0 ? 0 : -1);
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
    if (plan->probe_index >= 0) {  // locate the two captured event-record nodes
        size_t n = 0;
        hipGraphGetNodes(g, nullptr, &n);
        std::vector<hipGraphNode_t> nodes(n);
        hipGraphGetNodes(g, nodes.data(), &n);
        for (auto nd : nodes) {
            hipGraphNodeType t;
            if (hipGraphNodeGetType(nd, &t) != hipSuccess || t != hipGraphNodeTypeEventRecord) continue;
            hipEvent_t e = nullptr;
            hipGraphEventRecordNodeGetEvent(nd, &e);
            if (e == plan->ev0[0]) plan->node0 = nd;
            if (e == plan->ev1[0]) plan->node1 = nd;
        }
        if (!plan->node0 || !plan->node1) {
            plan->clear_graph();
            esm::set_error("plan: probe events were not captured as graph nodes");
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
