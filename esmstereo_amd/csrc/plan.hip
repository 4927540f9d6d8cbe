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
int launch_convt_1x1(const esm_conv_desc&, const esm_conv_desc&, hipStream_t);  // conv_up1.hip
int gwc_stem_check(const esm_conv_desc&, const float*, const float*, int, int);                // gwc_stem.hip
int launch_gwc_stem(const esm_conv_desc&, const float*, const float*, int, int, hipStream_t);  // gwc_stem.hip
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

enum OpKind { kConv = 1, kSmix = 2, kGwc = 3, kConcat = 4, kNormcorr = 5, kRegression = 6, kShuffleTail = 7, kFmnet = 9, kConf = 10, kShuffleConv = 12, kPair2 = 13, kGwcStem = 14, kConvt1x1 = 15 };

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
    int branch = 0;  // 0: the main chain; 1: the side branch (esm_plan_set_branch)
    int join = 0;    // main op: wait for the side ops listed before it (esm_plan_set_join)
};

int run_op(const Op& op, hipStream_t s) {
    switch (op.kind) {
        case kConv: return esm::launch_conv(&op.conv, s);
        case kSmix: return esm::launch_smix(&op.smix, s);
        case kFmnet: return esm::launch_fmnet(&op.fm, s);
        case kShuffleTail: return esm::launch_shuffle_tail(&op.st, s);
        case kShuffleConv: return esm::launch_shuffle_conv(&op.sc, s);
        case kPair2: return esm::conv::launch_pair2(op.conv, op.conv2, s);
        case kConvt1x1: return esm::conv::launch_convt_1x1(op.conv, op.conv2, s);
        case kConf: return esm::launch_conf(&op.cf, s);
        case kGwcStem: return esm::conv::launch_gwc_stem(op.conv, op.vol.L, op.vol.R, op.vol.C, op.vol.G, s);
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

// The kernel nodes captured for one op, in launch order: walk back from the capture frontier after
// the op to the frontier before it (the plan captures on one stream, so the graph is a chain).
std::vector<hipGraphNode_t> chain_between(const std::vector<hipGraphNode_t>& before,
                                          const std::vector<hipGraphNode_t>& after) {
    std::vector<hipGraphNode_t> out;
    if (after.size() != 1) return out;
    hipGraphNode_t nd = after[0];
    for (;;) {
        bool stop = false;
        for (auto b : before) stop = stop || (b == nd);
        if (stop) break;
        out.push_back(nd);
        size_t n = 0;
        if (hipGraphNodeGetDependencies(nd, nullptr, &n) != hipSuccess || n != 1) break;
        hipGraphNodeGetDependencies(nd, &nd, &n);
    }
    return std::vector<hipGraphNode_t>(out.rbegin(), out.rend());
}

// Every pointer field of an op that lies in one of the ranges [lo, hi) moves by that range's delta
// (the first range holding the ORIGINAL value: each field is looked at once, so swapped or chained
// bindings never move a pointer twice); returns how many moved.
struct Rebase {
    struct Range {
        uintptr_t lo, hi;
        intptr_t delta;
    };
    std::vector<Range> r;
    template <class T>
    int operator()(T*& p) const {
        const uintptr_t v = reinterpret_cast<uintptr_t>(p);
        if (!p) return 0;
        for (const Range& g : r) {
            if (v >= g.lo && v < g.hi) {
                p = reinterpret_cast<T*>(v + g.delta);
                return 1;
            }
        }
        return 0;
    }
    int conv(esm_conv_desc& d) const {
        int n = 0;
        for (int i = 0; i < d.nsrc && i < ESM_MAX_SRC; ++i) n += (*this)(d.src[i].ptr);
        n += (*this)(d.w) + (*this)(d.scale) + (*this)(d.shift) + (*this)(d.mul) + (*this)(d.res);
        return n + (*this)(d.out) + (*this)(d.up) + (*this)(d.out2) + (*this)(d.pre);
    }
    int stage(esm_smix_stage& t) const {
        return (*this)(t.ln_w) + (*this)(t.fc0_w) + (*this)(t.fc0_b) + (*this)(t.fc2_w) + (*this)(t.fc2_b);
    }
    int tail(esm_shuffle_tail_desc& t) const {
        return (*this)(t.x) + (*this)(t.up_w) + (*this)(t.up_b) + (*this)(t.tail_w) + (*this)(t.tail_b) + (*this)(t.out);
    }
};

}  // namespace

struct esm_plan {
    std::vector<Op> ops;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    hipStream_t cap_stream = nullptr;
    // the side branch: its stream and the fork / join events (created on first use)
    hipStream_t side_stream = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // probe
    int probe_index = -1;
    int ring = 0;
    std::vector<hipEvent_t> ev0, ev1;
    long long issued = 0, consumed = 0;
    hipGraphNode_t node0 = nullptr, node1 = nullptr;
    // per op: its kernel nodes in the captured graph (esm_plan_rebind updates them in place)
    std::vector<std::vector<hipGraphNode_t>> op_nodes;
    // recorded after every graph launch: a rebind waits on it before touching the instantiated graph
    hipEvent_t last_launch = nullptr;
    bool launched = false;

    void clear_graph() {
        if (exec) hipGraphExecDestroy(exec);
        if (graph) hipGraphDestroy(graph);
        exec = nullptr;
        graph = nullptr;
        node0 = node1 = nullptr;
        op_nodes.clear();
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
        if (last_launch) hipEventDestroy(last_launch);
        if (ev_fork) hipEventDestroy(ev_fork);
        if (ev_join) hipEventDestroy(ev_join);
        if (side_stream) hipStreamDestroy(side_stream);
        if (cap_stream) hipStreamDestroy(cap_stream);
    }
    bool has_side() const {
        for (const Op& op : ops)
            if (op.branch && op.repeat) return true;
        return false;
    }
    int side_setup() {
        if ((!side_stream && hipStreamCreateWithFlags(&side_stream, hipStreamNonBlocking) != hipSuccess) ||
            (!ev_fork && hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming) != hipSuccess) ||
            (!ev_join && hipEventCreateWithFlags(&ev_join, hipEventDisableTiming) != hipSuccess)) {
            esm::set_error("plan: cannot create the side-branch stream / events");
            return ESM_ERR_RUNTIME;
        }
        return ESM_OK;
    }
    // fork: the side stream continues from s's current point; join: s continues after the side stream's
    // last launch.  Under stream capture these are dependency edges, not nodes.
    int fork(hipStream_t s) {
        if (hipEventRecord(ev_fork, s) != hipSuccess || hipStreamWaitEvent(side_stream, ev_fork, 0) != hipSuccess) {
            esm::set_error("plan: side-branch fork failed");
            return ESM_ERR_RUNTIME;
        }
        return ESM_OK;
    }
    int joined(hipStream_t s) {
        if (hipEventRecord(ev_join, side_stream) != hipSuccess || hipStreamWaitEvent(s, ev_join, 0) != hipSuccess) {
            esm::set_error("plan: side-branch join failed");
            return ESM_ERR_RUNTIME;
        }
        return ESM_OK;
    }
    int patch(int i, const Rebase& rb) {
        Op& op = ops[i];
        switch (op.kind) {
            case kConv: return rb.conv(op.conv);
            case kPair2:
            case kConvt1x1: return rb.conv(op.conv) + rb.conv(op.conv2);
            case kGwcStem: return rb.conv(op.conv) + rb(op.vol.L) + rb(op.vol.R);
            case kSmix: {
                int n = rb(op.smix.x) + rb(op.smix.out) + rb(op.smix.res) + rb(op.smix.dw_w) + rb(op.smix.dw_b);
                for (int k = 0; k < op.smix.nstages && k < ESM_SMIX_MAX_STAGES; ++k) n += rb.stage(op.smix.stage[k]);
                return n;
            }
            case kFmnet: {
                int n = rb(op.fm.x) + rb(op.fm.out);
                for (int k = 0; k < 2; ++k) n += rb(op.fm.dw_w[k]) + rb(op.fm.dw_b[k]);
                for (int k = 0; k < 4; ++k) n += rb.stage(op.fm.stage[k]);
                return n + rb(op.fm.conv0_w) + rb(op.fm.conv0_b) + rb(op.fm.conv2_w) + rb(op.fm.conv2_b) + rb(op.fm.work);
            }
            case kShuffleTail: return rb.tail(op.st);
            case kShuffleConv:
                return rb.tail(op.sc.st) + rb(op.sc.w) + rb(op.sc.scale) + rb(op.sc.shift) + rb(op.sc.out) +
                       rb(op.sc.pre_x) + rb(op.sc.pre_w) + rb(op.sc.pre_scale) + rb(op.sc.pre_shift) + rb(op.sc.w2) +
                       rb(op.sc.scale2) + rb(op.sc.shift2);
            case kConf: {
                int n = rb(op.cf.out);
                for (int k = 0; k < 4; ++k) n += rb(op.cf.x[k]);
                return n;
            }
            case kGwc:
            case kConcat:
            case kNormcorr:
                return rb(op.vol.L) + rb(op.vol.R) + rb(op.vol.att) + rb(op.vol.V) + rb(op.vol.work);
            case kRegression: return rb(op.reg.cost) + rb(op.reg.out);
            default: return 0;
        }
    }
    // Re-capture op i alone and copy its kernel parameters into the instantiated graph's nodes of
    // that op.  False when the op's node structure changed (e.g. a source moved out of the window the
    // register-weight forms need, so the launcher picks another kernel): the caller rebuilds.
    bool refresh_op_nodes(int i) {
        if (i >= static_cast<int>(op_nodes.size())) return false;
        const std::vector<hipGraphNode_t>& nodes = op_nodes[i];
        if (nodes.empty()) return ops[i].repeat == 0;
        if (hipStreamBeginCapture(cap_stream, hipStreamCaptureModeThreadLocal) != hipSuccess) return false;
        int rc = ESM_OK;
        for (int r = 0; r < ops[i].repeat && rc == ESM_OK; ++r) rc = run_op(ops[i], cap_stream);
        hipGraph_t tg = nullptr;
        const hipError_t ec = hipStreamEndCapture(cap_stream, &tg);
        bool ok = rc == ESM_OK && ec == hipSuccess && tg;
        std::vector<hipGraphNode_t> tn;
        if (ok) {  // the temporary graph is a chain: roots, then successors
            std::vector<hipGraphNode_t> cur = graph_roots(tg);
            while (cur.size() == 1) {
                tn.push_back(cur[0]);
                cur = successors(cur);
            }
            ok = cur.empty() && tn.size() == nodes.size();
        }
        for (size_t k = 0; ok && k < tn.size(); ++k) {
            hipGraphNodeType ta, tb;
            ok = hipGraphNodeGetType(tn[k], &ta) == hipSuccess && hipGraphNodeGetType(nodes[k], &tb) == hipSuccess &&
                 ta == hipGraphNodeTypeKernel && tb == hipGraphNodeTypeKernel;
            hipKernelNodeParams p{}, q{};
            ok = ok && hipGraphKernelNodeGetParams(tn[k], &p) == hipSuccess &&
                 hipGraphKernelNodeGetParams(nodes[k], &q) == hipSuccess && p.func == q.func;
            ok = ok && hipGraphExecKernelNodeSetParams(exec, nodes[k], &p) == hipSuccess;
        }
        if (tg) hipGraphDestroy(tg);
        (void)hipGetLastError();
        return ok;
    }
    // Launch every op on s; when `slot` >= 0 record the probe pair `slot` around the probed op.
    // Under stream capture the records become event-record graph nodes (hipEventRecordExternal).
    int launch_all(hipStream_t s, int slot, bool capture = false) {
        const unsigned flags = capture ? hipEventRecordExternal : 0u;
        const bool side = has_side();
        bool pending = false;  // side launches not yet joined
        if (side) {
            int rc = side_setup();
            if (rc == ESM_OK) rc = fork(s);
            if (rc != ESM_OK) return rc;
        }
        for (int i = 0; i < static_cast<int>(ops.size()); ++i) {
            if (ops[i].branch) {
                for (int r = 0; r < ops[i].repeat; ++r) {
                    const int rc = run_op(ops[i], side_stream);
                    if (rc != ESM_OK) return rc;
                }
                pending = pending || ops[i].repeat > 0;
                continue;
            }
            if (ops[i].join && pending) {
                const int rc = joined(s);
                if (rc != ESM_OK) return rc;
                pending = false;
            }
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
        return side ? joined(s) : ESM_OK;  // (the side stream always rejoins: the run ends on s)
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
        case 9: return static_cast<int>(sizeof(esm_dwconv_desc));
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

int esm_plan_add_convt_1x1(esm_plan* plan, const esm_conv_desc* a, const esm_conv_desc* b) {
    if (!a || !b) return esm::arg_error("plan: null convt_1x1 desc");
    Op op;
    op.kind = kConvt1x1;
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

int esm_plan_add_gwc_stem(esm_plan* plan, const esm_conv_desc* stem, const float* L, const float* R, int C, int G) {
    if (!stem) return esm::arg_error("plan: null gwc_stem desc");
    const int rc = esm::conv::gwc_stem_check(*stem, L, R, C, G);
    if (rc != ESM_OK) return rc;
    Op op;
    op.kind = kGwcStem;
    op.conv = *stem;
    op.vol = VolArgs{L, R, nullptr, nullptr, nullptr, stem->B, C, stem->Hi, stem->Wi, stem->Di, G};
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

int esm_plan_set_branch(esm_plan* plan, int index, int branch) {
    if (!plan) return esm::arg_error("plan: null");
    if (index < 0 || index >= static_cast<int>(plan->ops.size())) return esm::arg_error("plan: op index out of range");
    if (branch != 0 && branch != 1) return esm::arg_error("plan: branch must be 0 (main) or 1 (side)");
    if (branch && index == plan->probe_index) return esm::arg_error("plan: the probed op must be on the main chain");
    plan->clear_graph();
    const int prev = plan->ops[index].branch;
    plan->ops[index].branch = branch;
    return prev;
}

int esm_plan_set_join(esm_plan* plan, int index, int join) {
    if (!plan) return esm::arg_error("plan: null");
    if (index < 0 || index >= static_cast<int>(plan->ops.size())) return esm::arg_error("plan: op index out of range");
    plan->clear_graph();
    const int prev = plan->ops[index].join;
    plan->ops[index].join = join ? 1 : 0;
    return prev;
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
    // Side-branch ops are captured on the side stream, forked from the capture's start and joined where a
    // main op asks (and at the end); each op's kernel nodes are found from its own stream's frontiers.
    std::vector<hipGraphNode_t> before, after;
    std::vector<std::vector<hipGraphNode_t>> frontiers;  // capture frontier (of the op's stream) after each op
    std::vector<std::vector<hipGraphNode_t>> prev_of;    // ... and before it
    const bool side = plan->has_side();
    int rc = side ? plan->side_setup() : ESM_OK;
    if (rc == ESM_OK && side) rc = plan->fork(plan->cap_stream);
    std::vector<hipGraphNode_t> last_main, last_side = capture_frontier(plan->cap_stream);
    last_main = last_side;
    bool pending = false;
    for (int i = 0; i < static_cast<int>(plan->ops.size()) && rc == ESM_OK; ++i) {
        const Op& op = plan->ops[i];
        if (op.branch) {
            prev_of.push_back(last_side);
            for (int r = 0; r < op.repeat && rc == ESM_OK; ++r) rc = run_op(op, plan->side_stream);
            last_side = capture_frontier(plan->side_stream);
            frontiers.push_back(last_side);
            pending = pending || op.repeat > 0;
            continue;
        }
        if (op.join && pending && rc == ESM_OK) {
            rc = plan->joined(plan->cap_stream);
            pending = false;
        }
        prev_of.push_back(last_main);
        if (i == plan->probe_index) before = capture_frontier(plan->cap_stream);
        for (int r = 0; r < op.repeat && rc == ESM_OK; ++r) rc = run_op(op, plan->cap_stream);
        last_main = capture_frontier(plan->cap_stream);
        frontiers.push_back(last_main);
        if (i == plan->probe_index) after = frontiers.back();
    }
    if (rc == ESM_OK && side) rc = plan->joined(plan->cap_stream);
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
    plan->op_nodes.resize(frontiers.size());
    for (size_t i = 0; i < frontiers.size(); ++i) plan->op_nodes[i] = chain_between(prev_of[i], frontiers[i]);
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
    if (!plan) return esm::arg_error("plan: null");
    if (!plan->exec) {  // never built, or dropped by a hint / repeat / probe change or a rebind
        const int rc = esm_plan_graph_build(plan, stream);
        if (rc != ESM_OK) return rc;
    }
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
    if (!plan->last_launch && hipEventCreateWithFlags(&plan->last_launch, hipEventDisableTiming) != hipSuccess) {
        esm::set_error("plan: hipEventCreate failed");
        return ESM_ERR_RUNTIME;
    }
    if (hipEventRecord(plan->last_launch, esm::as_stream(stream)) != hipSuccess) {
        esm::set_error("plan: hipEventRecord failed");
        return ESM_ERR_RUNTIME;
    }
    plan->launched = true;
    return ESM_OK;
}

int esm_plan_rebind(esm_plan* plan, int n, const void* const* old_base, const uint64_t* bytes,
                    const void* const* new_base) {
    if (!plan) return esm::arg_error("plan: null");
    if (n < 0 || (n > 0 && (!old_base || !bytes || !new_base))) return esm::arg_error("plan: bad rebind arrays");
    Rebase rb;
    for (int k = 0; k < n; ++k) {
        const uintptr_t lo = reinterpret_cast<uintptr_t>(old_base[k]);
        if (!old_base[k] || !new_base[k]) return esm::arg_error("plan: rebind of a null buffer");
        for (const Rebase::Range& g : rb.r)
            if (lo < g.hi && g.lo < lo + bytes[k]) return esm::arg_error("plan: rebind ranges overlap");
        rb.r.push_back({lo, lo + bytes[k], reinterpret_cast<intptr_t>(new_base[k]) - static_cast<intptr_t>(lo)});
    }
    std::vector<char> dirty(plan->ops.size(), 0);
    int moved = 0;
    for (size_t i = 0; i < plan->ops.size(); ++i) {
        const int m = plan->patch(static_cast<int>(i), rb);
        moved += m;
        dirty[i] = m > 0;
    }
    if (!plan->exec || !moved) return moved;
    // the instantiated graph's kernel arguments are about to change: the previous replay must have
    // finished reading them
    if (plan->launched && hipEventSynchronize(plan->last_launch) != hipSuccess) {
        plan->clear_graph();  // the ops moved but the nodes did not: rebuild from the ops at the next launch
        esm::set_error("plan: hipEventSynchronize failed");
        return ESM_ERR_RUNTIME;
    }
    for (size_t i = 0; i < dirty.size(); ++i) {
        if (dirty[i] && !plan->refresh_op_nodes(static_cast<int>(i))) {
            plan->clear_graph();  // rebuilt by the next esm_plan_graph_launch
            break;
        }
    }
    return moved;
}

int esm_plan_busy(esm_plan* plan) {
    if (!plan) return esm::arg_error("plan: null");
    if (!plan->launched) return 0;
    const hipError_t e = hipEventQuery(plan->last_launch);
    if (e == hipSuccess) return 0;
    if (e == hipErrorNotReady) return 1;
    esm::set_error("plan: hipEventQuery failed");
    return ESM_ERR_RUNTIME;
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
