// Network executor: GNN_lg / GNN_simple forward and backward as one enqueue.
//
// The reference runs every layer as Python-level torch ops with per-graph
// Python loops (models/gnns/model_mnb.py:58-66 GNN_simple.forward, 124-129
// GNN_lg.forward, order switch 102-119; models/layers/layers_mnb.py).
// Here the network is a fixed "program" of half-layers derived from the
// config: each half = aggregate (agg_fwd) -> fused Conv1d pair GEMM with
// bias/ReLU/BN-partials epilogue -> BN finalize -> BN apply.  The last layer is
// aggregate -> segmented readout.  Backward walks the program in reverse.  All
// activations live in one caller-provided workspace laid out here, so a
// forward+backward is a fixed sequence of launches with no allocation and no
// host synchronisation (graph-capturable).
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/hgnn_amd.h"
#include "kernels.h"

namespace hgnn {
namespace {

constexpr size_t ALIGN = 256;

struct Feat {
    bool edge;
    int c;
    size_t z = 0, y = 0, grad = 0;
    bool has_y = false;
};

struct Half {
    bool edge;
    int gin, pin;
    int cg, cp, k;
    int out, bn;
    int pw_lin, pb_lin, pw_relu, pb_relu, pbn_w, pbn_b;
    int relu_from;
    int kp;  // row stride of the dA buffer and logical width of the GEMM operand (k rounded up to 4: float4 k)
    bool id = false;  // diagonal I / D columns (AggFwdArgs::j0 = 2): the aggregate holds slices 2.. and P only
    int kpa = 0;      // row stride of the aggregate buffer: kp, or kp - 2 cg with id
    size_t a = 0, part = 0, mean = 0, stdv = 0;
    size_t wt = 0, wc = 0, bc = 0;  // repacked Conv1d-pair weights (repack.hip)
    size_t wc3 = 0;                 // Wcat as three bf16 planes [3][2d][bf3_ld(kp)] (split-bf16 forward GEMM)
    size_t bnf = 0;                 // the forward GEMM's BN sums by fp64 atomics [BN_ACC_COPIES][2][2d] (HGNN_BN_ACC)
    size_t wt3 = 0;                 // WT as three bf16 planes [3][k][bf3_ld(c2p)] (split-bf16 dA GEMM)
};

// Buffer ring of the backward: a dY / bias-partial buffer (and, for the node halves whose dense dW the side
// stream reads, a dA buffer) per half, up to this many halves, so the main stream never waits mid-backward
// for the side stream's dW of an earlier half before reusing a buffer (config 2: 8 halves, no such joins)
constexpr int BWD_NBUF = 16;

struct Program {
    int cap_n = 0, cap_e = 0, jt = 0, d = 0, c2 = 0;
    int c2p = 0;  // 2d rounded up to 4: row stride of dY and of the repacked WT (dA GEMM's float4 k)
    int n_params = 0, n_bn = 0;
    std::vector<Feat> feats;
    std::vector<Half> halves;
    int last_gin = -1, last_pin = -1, k_last = 0, p_fcw = 0, p_fcb = 0;
    size_t a_last = 0, colsum = 0;
    size_t diag_n = 0, diag_e = 0;  // per row (v_0, v_1) of the diagonal operator entry (diagonal I / D mode)
    size_t node_off = 0, edge_off = 0, totals = 0, err = 0;
    size_t rows[S_COUNT] = {}, ent[S_COUNT] = {};
    int entry_stride_w = 4;
    size_t da = 0, slabs = 0, bnb_part = 0, bnb_sums = 0, rb_scratch = 0;
    size_t bnb_acc[2] = {};  // BN-backward statistics accumulators (BnBwdArgs::acc64), ping-pong over the walk
    size_t acc_end = 0;      // end of the accumulator run (bnb_acc[0] .. the halves' bnf, the forward ticket)
    size_t fwd_ticket = 0;  // the forward GEMM's last-block finalize (FwdBnFin)
    int nbuf = 0;  // ring length: min(halves, BWD_NBUF)
    size_t dyk[BWD_NBUF] = {}, dbk[BWD_NBUF] = {}, dak[BWD_NBUF] = {};
    size_t bytes = 0;
};

struct Bump {
    size_t top = 0;
    size_t take(size_t n) {
        const size_t o = top;
        top += (n + ALIGN - 1) / ALIGN * ALIGN;
        return o;
    }
};

bool valid_config(const hgnn_net_config* c) {
    if (!c) return false;
    if (c->kind != 0 && c->kind != 1) return false;
    if (c->bs <= 0 || c->nmax <= 0 || c->f_in <= 0 || c->d <= 0 || c->n_layers < 2) return false;
    if (c->dim_out <= 0) return false;
    if (c->kind == 1 && (c->emax < 0 || c->order < 1 || c->order > 3)) return false;
    if (c->j_tot < 3 || c->j_tot > 7) return false;  // entries of 8 floats: column + up to 7 slices
    if (2 * c->d > 512) return false;
    const long long capn = (long long)c->bs * c->nmax;
    const long long cape = (long long)c->bs * (c->kind == 1 ? c->emax : 0);
    if (capn * c->nmax > (1ll << 31) - 1) return false;
    if (cape * (c->emax > c->nmax ? c->emax : c->nmax) > (1ll << 31) - 1) return false;
    return true;
}

static bool env_flag(const char* name, bool dflt) {
    const char* e = getenv(name);
    if (!e || !e[0]) return dflt;
    return e[0] != '0';
}

// The forward Conv1d-pair GEMM on bf16 MFMA with three-way split operands (gemm_bf3.hip: fp32 accuracy,
// 2.7x fewer MFMA cycles); HGNN_FWD_BF3=0: the fp32 MFMA kernels (launch_gemm3_fwd).  Line-graph networks
// with 2d % 64 == 0 (the kernel's 64-column tiles).
static bool fwd_bf3_c2(int c2) {
    static const bool on = env_flag("HGNN_FWD_BF3", true);
    return on && c2 % 64 == 0;
}
// Diagonal I / D columns (round 6; HGNN_DIAG_ID=1: on, off by default -- measured 1.110 vs 1.105 ms per step in three
// of three alternating pairs at config 2: the aggregation lost 5 us per step, the forward and dW GEMMs' staging
// gained 11 and 14): graph_operators' slices 0 and 1 are I and diag(D)
// (functions/operators.py:19-23), so the aggregate's I / D column blocks are x̂ and D_r x̂ -- two of the five
// column blocks of a line-graph half at J = 1, written by the aggregation and read by the forward and dW GEMMs.
// In this mode the aggregation stores only slices 2.. and P (plus each row's diagonal coefficients) and the two
// split-bf16 GEMMs build the I / D columns from the half's input x̂ as they stage it (DiagIdArgs), the same
// values bit for bit.  For the halves whose G input is a BN'd layer output of 2d <= 256 channels (not the
// raw inputs of layer 0), with the split-bf16 forward and dW GEMMs.
static bool diag_id_on(int c2) {
    static const bool on = env_flag("HGNN_DIAG_ID", false);
    return on && fwd_bf3_c2(c2) && dw_bf3_enabled() && c2 <= 256;
}

Program build_program(const hgnn_net_config* c) {
    Program P;
    const bool lg = c->kind == 1;
    P.cap_n = c->bs * c->nmax;
    P.cap_e = lg ? c->bs * c->emax : 0;
    P.jt = c->j_tot;
    P.d = c->d;
    P.c2 = 2 * c->d;
    P.c2p = (P.c2 + 3) / 4 * 4;
    P.entry_stride_w = c->j_tot <= 3 ? 4 : 8;
    const int L = c->n_layers;
    P.n_params = (lg ? 12 : 6) * (L - 1) + 2;
    P.n_bn = (lg ? 2 : 1) * (L - 1);

    auto add_feat = [&](bool edge, int ch) {
        Feat f;
        f.edge = edge;
        f.c = ch;
        P.feats.push_back(f);
        return (int)P.feats.size() - 1;
    };
    add_feat(false, c->f_in);
    if (lg) add_feat(true, 1);
    int in_n = 0, in_e = lg ? 1 : -1;
    for (int l = 0; l < L - 1; ++l) {
        if (lg) {
            const int pb = 12 * l;
            const int out_n = add_feat(false, P.c2);
            const int out_e = add_feat(true, P.c2);
            P.feats[out_n].has_y = P.feats[out_e].has_y = true;
            Half hn{}, he{};
            hn.edge = false;
            hn.gin = in_n;
            hn.cg = P.feats[in_n].c;
            hn.out = out_n;
            hn.bn = 2 * l;
            hn.pw_relu = pb + 0;
            hn.pb_relu = pb + 1;
            hn.pw_lin = pb + 2;
            hn.pb_lin = pb + 3;
            hn.pbn_w = pb + 4;
            hn.pbn_b = pb + 5;
            hn.relu_from = c->d;
            he.edge = true;
            he.gin = in_e;
            he.cg = P.feats[in_e].c;
            he.out = out_e;
            he.bn = 2 * l + 1;
            he.pw_relu = pb + 6;
            he.pb_relu = pb + 7;
            he.pw_lin = pb + 8;
            he.pb_lin = pb + 9;
            he.pbn_w = pb + 10;
            he.pbn_b = pb + 11;
            he.relu_from = c->d;
            if (c->order == 1) {  // node first; edge half reads the BN'd node output
                hn.pin = in_e;
                he.pin = out_n;
            } else if (c->order == 2) {  // edge first; node half reads the BN'd edge output
                he.pin = in_n;
                hn.pin = out_e;
            } else {  // independent halves
                hn.pin = in_e;
                he.pin = in_n;
            }
            hn.cp = P.feats[hn.pin].c;
            he.cp = P.feats[he.pin].c;
            hn.k = P.jt * hn.cg + 2 * hn.cp;
            he.k = P.jt * he.cg + 2 * he.cp;
            if (c->order == 2) {
                P.halves.push_back(he);
                P.halves.push_back(hn);
            } else {
                P.halves.push_back(hn);
                P.halves.push_back(he);
            }
            in_n = out_n;
            in_e = out_e;
        } else {
            const int pb = 6 * l;
            const int out_n = add_feat(false, P.c2);
            P.feats[out_n].has_y = true;
            Half h{};
            h.edge = false;
            h.gin = in_n;
            h.cg = P.feats[in_n].c;
            h.pin = -1;
            h.cp = 0;
            h.k = P.jt * h.cg;
            h.out = out_n;
            h.bn = l;
            // layer_simple: cat(relu(cv2(x)), relu(cv1(x))) -> both halves ReLU (layers_mnb.py:59-65)
            h.pw_lin = pb + 2;
            h.pb_lin = pb + 3;
            h.pw_relu = pb + 0;
            h.pb_relu = pb + 1;
            h.pbn_w = pb + 4;
            h.pbn_b = pb + 5;
            h.relu_from = 0;
            P.halves.push_back(h);
            in_n = out_n;
        }
    }
    for (Half& h : P.halves) {
        bool prod = false;
        for (const Half& o : P.halves) prod = prod || o.out == h.gin;
        h.id = diag_id_on(P.c2) && prod && h.cg == P.c2 && (h.pin < 0 || h.cp == P.c2);
    }
    P.last_gin = in_n;
    P.last_pin = lg ? in_e : -1;
    P.k_last = P.jt * P.feats[in_n].c + (lg ? 2 * P.feats[in_e].c : 0);
    P.p_fcw = P.n_params - 2;
    P.p_fcb = P.n_params - 1;

    // ---- workspace layout
    Bump B;
    P.node_off = B.take(sizeof(int) * (c->bs + 1));
    P.edge_off = B.take(sizeof(int) * (c->bs + 1));
    P.totals = B.take(sizeof(int) * 4);
    P.err = B.take(sizeof(uint32_t) * 4);
    const int nmax = c->nmax, emax = lg ? c->emax : 0;
    const size_t sw = P.entry_stride_w * sizeof(float);
    P.rows[S_W] = B.take(sizeof(RowInfo) * P.cap_n);
    P.ent[S_W] = B.take((size_t)P.cap_n * nmax * sw);
    P.rows[S_WT] = B.take(sizeof(RowInfo) * P.cap_n);
    P.ent[S_WT] = B.take((size_t)P.cap_n * nmax * sw);
    if (lg) {
        P.rows[S_WL] = B.take(sizeof(RowInfo) * P.cap_e);
        P.ent[S_WL] = B.take((size_t)P.cap_e * emax * sw);
        P.rows[S_WLT] = B.take(sizeof(RowInfo) * P.cap_e);
        P.ent[S_WLT] = B.take((size_t)P.cap_e * emax * sw);
        P.rows[S_PN] = B.take(sizeof(RowInfo) * P.cap_n);
        P.ent[S_PN] = B.take((size_t)P.cap_n * emax * 16);
        P.rows[S_PE] = B.take(sizeof(RowInfo) * P.cap_e);
        P.ent[S_PE] = B.take((size_t)P.cap_e * nmax * 16);
    }
    for (auto& f : P.feats) {
        const size_t cap = f.edge ? P.cap_e : P.cap_n;
        if (f.has_y) f.y = B.take(cap * f.c * sizeof(float));
        else f.z = B.take(cap * f.c * sizeof(float));
        f.grad = B.take(cap * f.c * sizeof(float));
    }
    size_t max_da = 0, max_slab = 0;
    int max_cap = 0;
    for (auto& h : P.halves) {
        const int cap = h.edge ? P.cap_e : P.cap_n;
        h.kp = (h.k + 3) / 4 * 4;
        h.kpa = h.id ? h.kp - 2 * h.cg : h.kp;
        h.a = B.take((size_t)cap * h.kpa * sizeof(float));
        h.part = B.take((size_t)gemm_fwd_tiles_m(cap) * P.c2 * 3 * sizeof(float));
        h.mean = B.take(P.c2 * sizeof(float));
        h.stdv = B.take(P.c2 * sizeof(float));
        h.wt = B.take((size_t)h.k * P.c2p * sizeof(float));
        h.wc = B.take((size_t)P.c2 * h.kp * sizeof(float));
        h.bc = B.take((size_t)P.c2 * sizeof(float));
        h.wc3 = B.take((size_t)3 * P.c2 * bf3_ld(h.kp) * 2);
        h.wt3 = B.take((size_t)3 * h.k * bf3_ld(P.c2p) * 2);
        max_da = std::max(max_da, (size_t)cap * h.kp);
        max_slab = std::max(max_slab, dw3_slab_floats(cap, P.c2, h.k));
        max_cap = std::max(max_cap, cap);
    }
    // ring slot q % nbuf for the q-th half of the backward's walk (the last half first)
    P.nbuf = std::max(1, std::min((int)P.halves.size(), BWD_NBUF));
    for (int i = 0; i < P.nbuf; ++i) {
        P.dbk[i] = B.take((size_t)bn_bwd_tiles(max_cap > 0 ? max_cap : 1) * P.c2 * sizeof(float));
        P.dyk[i] = B.take((size_t)max_cap * P.c2p * sizeof(float));
        size_t na = 0;  // the node halves of this slot (their dA is read by the side stream's dense dW)
        for (int q = i; q < (int)P.halves.size(); q += P.nbuf) {
            const Half& h = P.halves[P.halves.size() - 1 - q];
            if (!h.edge) na = std::max(na, (size_t)P.cap_n * h.kp);
        }
        if (na) P.dak[i] = B.take(na * sizeof(float));
    }
    P.diag_n = B.take((size_t)P.cap_n * sizeof(float2));
    if (lg) P.diag_e = B.take((size_t)P.cap_e * sizeof(float2));
    P.a_last = B.take((size_t)P.cap_n * P.k_last * sizeof(float));
    P.colsum = B.take((size_t)c->bs * P.k_last * sizeof(float));
    max_da = std::max(max_da, (size_t)P.cap_n * P.k_last);
    P.da = B.take(max_da * sizeof(float));  // dA of the halves the side stream does not read, and the readout's
    P.slabs = B.take(max_slab * sizeof(float));
    P.bnb_part = B.take((size_t)bn_bwd_tiles(max_cap) * P.c2 * 4 * sizeof(float));
    // the statistics accumulators, one contiguous run zeroed by the forward's first kernel: the backward's two
    // ping-pong regions, then one forward region per half
    for (int i = 0; i < 2; ++i) P.bnb_acc[i] = B.take((size_t)bn_acc_doubles(P.c2) * sizeof(double));
    for (auto& h : P.halves) h.bnf = B.take((size_t)BN_ACC_COPIES * 2 * P.c2 * sizeof(double));
    P.fwd_ticket = B.take(sizeof(unsigned));
    P.acc_end = B.top;
    P.bnb_sums = B.take((size_t)P.c2 * 4 * sizeof(float));
    P.rb_scratch = B.take(readout_bwd_scratch_bytes(c->dim_out, P.k_last));
    P.bytes = B.top;
    return P;
}

// Program of a configuration, cached per host thread: built four times per training step
// otherwise (workspace query, forward, error word, backward), vectors included.
const Program& program_of(const hgnn_net_config* c) {
    struct Entry {
        int key[11];
        Program P;
    };
    thread_local std::vector<Entry> cache;
    const int key[11] = {c->kind, c->order, c->bs, c->nmax, c->emax, c->f_in, c->d, c->n_layers, c->j_tot,
                         c->dim_out, c->training};
    for (const Entry& e : cache)
        if (memcmp(e.key, key, sizeof(key)) == 0) return e.P;
    if (cache.size() >= 16) cache.erase(cache.begin());
    cache.push_back(Entry{});
    memcpy(cache.back().key, key, sizeof(key));
    cache.back().P = build_program(c);
    return cache.back().P;
}

// The GEMMs address each operand through a 32-bit buffer resource: every operand the
// program hands them must stay under 2 GB (checked before anything is enqueued).
bool fits_32bit(const Program& P) {
    const long long lim = (1ll << 31) - 1;
    for (const Half& h : P.halves) {
        const long long cap = h.edge ? P.cap_e : P.cap_n;
        if (cap * h.kp * 4 > lim || cap * P.c2p * 4 > lim || (long long)P.c2p * h.kp * 4 > lim) return false;
    }
    return (long long)P.cap_n * P.k_last * 4 <= lim;
}

template <typename T>
T* at(void* ws, size_t off) {
    return reinterpret_cast<T*>(static_cast<char*>(ws) + off);
}

// A layer output is kept pre-BN (y) only; its readers apply the BN of the half
// that produced it on load (BnView).  Inputs (feature 0, XL) are stored as is.
const Half* producer(const Program& P, int f) {
    for (const Half& h : P.halves)
        if (h.out == f) return &h;
    return nullptr;
}

const float* feat_src(const Program& P, void* ws, int f, const float* x0 = nullptr, const float* xl0 = nullptr) {
    if (f == 0 && x0) return x0;
    if (f == 1 && xl0 && P.feats[1].edge && !P.feats[1].has_y) return xl0;
    return P.feats[f].has_y ? at<float>(ws, P.feats[f].y) : at<float>(ws, P.feats[f].z);
}

BnView feat_bn(const Program& P, void* ws, const float* const* prm, int f) {
    BnView v{};
    const Half* h = producer(P, f);
    if (!h) return v;
    v.mean = at<float>(ws, h->mean);
    v.std = at<float>(ws, h->stdv);
    v.w = prm[h->pbn_w];
    v.b = prm[h->pbn_b];
    return v;
}

// The diagonal I / D operand of a half's GEMMs (DiagIdArgs): its G input (pre-BN y, BN on load) and the row
// coefficients of its kind
DiagIdArgs diag_id_args(const Program& P, void* ws, const float* const* prm, const Half& h) {
    DiagIdArgs d{};
    if (!h.id) return d;
    d.x = feat_src(P, ws, h.gin);
    d.ldx = P.feats[h.gin].c;
    d.c = h.cg;
    d.diag = at<float2>(ws, h.edge ? P.diag_e : P.diag_n);
    d.bn = feat_bn(P, ws, prm, h.gin);
    return d;
}

// Where a call's batch structure lives: the workspace (filled by the device
// extraction from the dense inputs) or a CSR batch image built on the host.
struct Src {
    BatchMeta m;
    StructView v[S_COUNT];
    const float* x0 = nullptr;   // packed node input (CSR batch) -- else feats[0].z
    const float* xl0 = nullptr;  // packed edge input (CSR batch) -- else feats[1].z
    long long nodes = 0;         // host node count (CSR batch)
};

BatchMeta meta_of(const Program& P, void* ws) {
    BatchMeta m;
    m.node_off = at<int>(ws, P.node_off);
    m.edge_off = at<int>(ws, P.edge_off);
    m.totals = at<int>(ws, P.totals);
    m.err = at<uint32_t>(ws, P.err);
    return m;
}

StructView view(const Program& P, void* ws, int kind) {
    StructView v;
    v.rows = at<RowInfo>(ws, P.rows[kind]);
    v.entries = at<float>(ws, P.ent[kind]);
    v.stride = (kind == S_PN || kind == S_PE) ? 4 : P.entry_stride_w;
    return v;
}

Src make_src(const Program& P, void* ws, const hgnn_csr_batch* csr) {
    Src r;
    r.m = meta_of(P, ws);
    for (int k = 0; k < S_COUNT; ++k) r.v[k] = view(P, ws, k);
    if (csr) {
        r.m.node_off = const_cast<int*>(static_cast<const int*>(csr->d_node_off));
        r.m.edge_off = const_cast<int*>(static_cast<const int*>(csr->d_edge_off));
        r.m.totals = const_cast<int*>(static_cast<const int*>(csr->d_totals));
        for (int k = 0; k < S_COUNT; ++k) {
            r.v[k].rows = static_cast<const RowInfo*>(csr->d_rows[k]);
            r.v[k].entries = csr->d_entries[k];
            r.v[k].stride = (k == S_PN || k == S_PE) ? 4 : csr->stride_w;
        }
        r.x0 = csr->d_x;
        r.xl0 = csr->d_xl;
        r.nodes = csr->nodes;
    }
    return r;
}

#define TRY(x)                  \
    do {                        \
        int _r = (x);           \
        if (_r) return _r;      \
    } while (0)

// Optional per-kernel-class timer (bench.py times the dominant kernel class and the aggregation classes
// inside their timed regions with it).  Disabled (nullptr) on the normal path.  Modes (hgnn_timer_create_ex):
//   HGNN_TIMER_STAMPS     the launches of the timed classes that carry a stamp slot (the aggregation and GEMM
//                         kernels) write s_memrealtime per wave at entry and exit (common.h WaveStamp); a
//                         launch's time = max(exit) - min(entry).  Nothing is added to the stream, so the timed
//                         kernel runs as in an untimed step.
//   HGNN_TIMER_DISPATCH   every dispatch of a timed class gets an event pair bound to the dispatch itself
//                         (hipExtLaunchKernel); every class is covered, but a timed dispatch runs slower (its
//                         completion signal's system-scope release: 19 -> 30 us per aggregation-backward launch
//                         inside rocprofv3's own trace).
//   HGNN_TIMER_MARKERS    marker events recorded on the stream around each call (the round-1..4 form).
struct Timer {
    std::vector<hipEvent_t> ev;   // pairs: start, stop
    std::vector<int> cls;
    int used = 0;
    unsigned mask = 0;
    int mode = HGNN_TIMER_DISPATCH;
    uint64_t* st = nullptr;  // stamp buffer (device)
    long long st_cap = 0, st_used = 0;
    std::vector<int> st_off, st_n;
    std::vector<uintptr_t> st_strm;
    std::vector<double> st_ms;  // per launch, filled on the first read after a region
    std::vector<uint64_t> st_lo, st_hi;  // per launch: first entry / last exit stamp (10 ns ticks)
    bool st_read = false;
    int rd_used = -1;         // used / st_used at the last read: a read is reused only while neither moved
    long long rd_st_used = -1;
};

struct ClockScope {  // t_clock for the launches of one TL call
    LaunchClock c;
    LaunchClock* prev;
    ClockScope(Timer* tm, int k, hipStream_t s) : prev(t_clock) {
        c = LaunchClock{};
        c.cls = tm->cls.data();
        c.cap = (int)tm->cls.size();
        c.used = &tm->used;
        c.k = k;
        if (tm->mode == HGNN_TIMER_STAMPS) {
            c.st = tm->st;
            c.st_off = tm->st_off.data();
            c.st_n = tm->st_n.data();
            c.st_cap = tm->st_cap;
            c.st_used = &tm->st_used;
            c.strm = reinterpret_cast<uintptr_t>(s);
            c.st_strm = tm->st_strm.data();
        } else {
            c.ev = tm->ev.data();
        }
        t_clock = &c;
    }
    ~ClockScope() { t_clock = prev; }
};

#define TL(k, x)                                                                        \
    do {                                                                                \
        const bool _t = tm && (tm->mask & (1u << (k))) && tm->used < (int)tm->cls.size(); \
        if (_t && tm->mode != HGNN_TIMER_MARKERS) {                                     \
            ClockScope _cs(tm, (k), s);                                                    \
            int _r = (x);                                                               \
            if (_r) return _r;                                                          \
            break;                                                                      \
        }                                                                               \
        if (_t) HGNN_HOST_CHECK(hipEventRecord(tm->ev[2 * tm->used], s));                \
        int _r = (x);                                                                   \
        if (_r) return _r;                                                              \
        if (_t) {                                                                       \
            HGNN_HOST_CHECK(hipEventRecord(tm->ev[2 * tm->used + 1], s));                \
            tm->cls[tm->used++] = (k);                                                  \
        }                                                                               \
    } while (0)

// Side stream.  Backward: the weight-gradient GEMM of a half (and its slab
// reduction) only feeds the parameter grads, so it runs beside the dA -> dense dW
// -> aggregation-backward chain of the same half.  Fork after the half's BN
// backward, join before the next half's BN backward overwrites dY / the bias
// partials, and once more at the end.  One non-blocking stream and a few events
// per host thread and device, created on first use.
struct SideStream {
    int dev = -1;
    hipStream_t s = nullptr;
    hipEvent_t fork[2] = {nullptr, nullptr}, join[BWD_NBUF + 1] = {};  // join[BWD_NBUF]: the end of the backward
};

static int side_stream(hipStream_t main_s, SideStream** out) {
    thread_local SideStream ss;
    // the device the caller's stream belongs to, not the thread's current device: the side
    // stream's kernels read and write the main stream's buffers
    hipDevice_t dev = 0;
    HGNN_HOST_CHECK(hipStreamGetDevice(main_s, &dev));
    if (ss.dev != dev) {
        int cur = 0;
        HGNN_HOST_CHECK(hipGetDevice(&cur));
        HGNN_HOST_CHECK(hipSetDevice(dev));
        if (ss.s) {
            (void)hipStreamDestroy(ss.s);
            for (int i = 0; i < 2; ++i) (void)hipEventDestroy(ss.fork[i]);
            for (int i = 0; i <= BWD_NBUF; ++i) (void)hipEventDestroy(ss.join[i]);
        }
        ss = SideStream{};
        // (the HIP runtime maps a process's streams round-robin onto GPU_MAX_HW_QUEUES hardware queues: with an RCCL
        // process group's streams this one can land on the main stream's queue and run serialised with it -- 8 queues
        // avoid it; a high- or low-priority side stream made the host's launches slow, round 6)
        HGNN_HOST_CHECK(hipStreamCreateWithFlags(&ss.s, hipStreamNonBlocking));
        // fork / join events without the system-scope fence of a record (hipEventDisableSystemFence): the two
        // streams are on one device, so the producing kernel's end-of-kernel release and the consumer's
        // dispatch acquire already order the data, and the fence's cache writeback / invalidate only delays
        // the main stream's next kernel -- 1.163-1.169 vs 1.193-1.197 ms per step in three alternating pairs
        // (profiles/r05_ab_event_fence.txt); HGNN_EVENT_FENCE=1 restores the fenced records
        static const bool fence = env_flag("HGNN_EVENT_FENCE", false);
        const unsigned ef = hipEventDisableTiming | (fence ? 0u : hipEventDisableSystemFence);
        for (int i = 0; i < 2; ++i) HGNN_HOST_CHECK(hipEventCreateWithFlags(&ss.fork[i], ef));
        for (int i = 0; i < BWD_NBUF; ++i) HGNN_HOST_CHECK(hipEventCreateWithFlags(&ss.join[i], ef));
        // the end-of-backward join hands the side stream's final dW / bias gradients to the caller's stream,
        // whose next consumer may be a D2H copy (gloo DP) or a peer: that record keeps the system-scope
        // release (once per step)
        HGNN_HOST_CHECK(hipEventCreateWithFlags(&ss.join[BWD_NBUF], hipEventDisableTiming));
        ss.dev = dev;
        HGNN_HOST_CHECK(hipSetDevice(cur));
    }
    *out = &ss;
    return 0;
}

static bool fwd_bf3(const Program& P) { return fwd_bf3_c2(P.c2); }
// BN-backward statistics by fp64 atomics into accumulator copies, no k_bn_bwd_fin (round 6; HGNN_BN_ACC=0: the
// per-tile partials and k_bn_bwd_fin).  The sums' order over the tiles is not fixed: the statistics can differ in the
// last fp64 bits from run to run (a float flip of m1 / m2 once in ~1e9 values), where the fin path is bitwise
// deterministic.
static bool bn_acc_on() {
    static const bool on = env_flag("HGNN_BN_ACC", true);
    return on;
}
// the forward BN finalize in the forward GEMM's last block (FwdBnFin; HGNN_BN_FWD_FIN=0: k_bn_finalize): 1.093 vs
// 1.106 ms median, five of five alternating pairs
static bool bn_fwd_fin_on() {
    static const bool on = env_flag("HGNN_BN_FWD_FIN", true);
    return on;
}
// The forward's first kernel zeroes both accumulator regions (k_plan; a CSR batch: the error word's memset)
static void bn_acc_zero_meta(const Program& P, void* ws, BatchMeta& m) {
    if (!bn_acc_on()) return;
    m.zero64 = at<double>(ws, P.bnb_acc[0]);
    m.zero64_n = (int)((P.acc_end - P.bnb_acc[0]) / sizeof(double));
}
// the dA GEMM on the split-bf16 kernel (k_gemm_bf3_fwd with a plain-store epilogue, B = WT's planes)
static bool da_bf3(const Program& P) {
    static const bool on = env_flag("HGNN_DA_BF3", true);
    return on && P.c2p <= 128;
}

int net_forward(const hgnn_net_config* c, const hgnn_net_inputs* in, const hgnn_csr_batch* csr,
                const float* const* prm, float* const* run, void* ws, float* out, hipStream_t s, Timer* tm) {
    const Program& P = program_of(c);
    if (!fits_32bit(P)) return HGNN_ERR_UNSUPPORTED;
    const bool lg = c->kind == 1;
    const Src src = make_src(P, ws, csr);
    BatchMeta m = src.m;
    std::vector<RepackTable> tables;
    {
        RepackTable rt{};
        rt.d = P.d;
        for (size_t hi = 0; hi < P.halves.size(); ++hi) {
            const Half& h = P.halves[hi];
            RepackItem& it = rt.it[rt.n++];
            it.wl = prm[h.pw_lin];
            it.wr = prm[h.pw_relu];
            it.bl = prm[h.pb_lin];
            it.br = prm[h.pb_relu];
            it.wt = at<float>(ws, h.wt);
            it.wc = at<float>(ws, h.wc);
            it.bc = at<float>(ws, h.bc);
            it.k = h.k;
            it.kp = h.kp;
            it.ldt = P.c2p;
            if (fwd_bf3(P)) {
                it.wc3 = at<__bf16>(ws, h.wc3);
                it.ldc3 = bf3_ld(h.kp);
            }
            if (da_bf3(P)) {
                it.wt3 = at<__bf16>(ws, h.wt3);
                it.ldt3 = bf3_ld(P.c2p);
            }
            if (rt.n == REPACK_MAX || hi + 1 == P.halves.size()) {
                tables.push_back(rt);
                rt.n = 0;
            }
        }
    }
    size_t plan_tables = 0;
    bn_acc_zero_meta(P, ws, m);
    if (csr) {  // dense inputs: k_plan zeroes both
        HGNN_HOST_CHECK(hipMemsetAsync(m.err, 0, sizeof(uint32_t), s));
        if (m.zero64) HGNN_HOST_CHECK(hipMemsetAsync(m.zero64, 0, (size_t)m.zero64_n * sizeof(double), s));
    }
    if (!csr) {
    plan_tables = tables.empty() ? 0 : 1;
    TL(HGNN_K_STRUCT, launch_plan(in->d_N_batch, lg ? in->d_E_batch : nullptr, c->bs, c->nmax, lg ? c->emax : 0, m, s,
                                  tables.empty() ? nullptr : &tables[0]));

    ExtractArgs ex{};
    ex.W = in->d_W;
    ex.WL = in->d_WL;
    ex.Pm = in->d_Pm;
    ex.Pd = in->d_Pd;
    ex.mask = in->d_mask;
    ex.mask_lg = in->d_mask_lg;
    ex.bs = c->bs;
    ex.nmax = c->nmax;
    ex.emax = lg ? c->emax : 0;
    ex.jtot = c->j_tot;
    ex.meta = m;
    for (int k = 0; k < S_COUNT; ++k) {
        ex.rows[k] = at<RowInfo>(ws, P.rows[k]);
        ex.entries[k] = at<float>(ws, P.ent[k]);
    }
    ex.entry_stride_w = P.entry_stride_w;
    ex.validate = 1;
    ex.dual = lg ? 1 : 0;
    ex.X = in->d_X;
    ex.f = c->f_in;
    ex.xo = at<float>(ws, P.feats[0].z);
    if (lg) {
        ex.XL = in->d_XL;
        ex.xlo = at<float>(ws, P.feats[1].z);
    }
    TL(HGNN_K_STRUCT, launch_extract(ex, s));
    }

    const int* tot_n = m.totals;
    const int* tot_e = m.totals + 1;
    // the repack tables of the Conv1d pairs of every half: Wcat^T (forward B) and padded Wcat (dA B);
    // the first rides in k_plan's launch (dense inputs), the rest (> REPACK_MAX halves, or a CSR
    // batch) are launches of their own
    for (size_t t = plan_tables; t < tables.size(); ++t) TL(HGNN_K_STRUCT, launch_repack(tables[t], s));
    for (int hi = 0; hi < (int)P.halves.size(); ++hi) {
        const Half& h = P.halves[hi];
        const int cap = h.edge ? P.cap_e : P.cap_n;
        const int* tot = h.edge ? tot_e : tot_n;
        AggFwdArgs ag{};
        ag.total_rows = tot;
        ag.cap_rows = cap;
        ag.g = src.v[h.edge ? S_WL : S_W];
        ag.xg = feat_src(P, ws, h.gin, src.x0, src.xl0);
        ag.gbn = feat_bn(P, ws, prm, h.gin);
        ag.cg = h.cg;
        ag.jtot = P.jt;
        if (h.pin >= 0) {
            ag.p = src.v[h.edge ? S_PE : S_PN];
            ag.xp = feat_src(P, ws, h.pin, src.x0, src.xl0);
            ag.pbn = feat_bn(P, ws, prm, h.pin);
            ag.cp = h.cp;
        }
        ag.out = at<float>(ws, h.a);
        ag.ldo = h.kpa;
        if (h.id) {
            ag.j0 = 2;
            // the first diagonal-I / D half of its kind records the rows' diagonal coefficients
            bool first = true;
            for (int q = 0; q < hi; ++q) first = first && !(P.halves[q].id && P.halves[q].edge == h.edge);
            if (first) {
                ag.diag = at<float2>(ws, h.edge ? P.diag_e : P.diag_n);
                ag.err = m.err;
            }
        }
        TL(HGNN_K_AGG_FWD, launch_agg_fwd(ag, s));

        const DiagIdArgs ida = diag_id_args(P, ws, prm, h);
        // the BN statistics by fp64 atomics (split-bf16 forward GEMM, training)
        double* bnf = fwd_bf3(P) && c->training && bn_acc_on() ? at<double>(ws, h.bnf) : nullptr;
        FwdBnFin fbn{};
        const bool gfin = bnf && bn_fwd_fin_on();
        if (gfin) {
            fbn.mean = at<float>(ws, h.mean);
            fbn.std = at<float>(ws, h.stdv);
            fbn.run_mean = run ? run[2 * h.bn] : nullptr;
            fbn.run_std = run ? run[2 * h.bn + 1] : nullptr;
            fbn.momentum = 0.1f;
            fbn.ticket = at<unsigned>(ws, P.fwd_ticket);
        }
        if (fwd_bf3(P))
            TL(HGNN_K_GEMM_FWD, launch_gemm_bf3_fwd(at<float>(ws, h.a), h.kpa, tot, cap, h.kp, at<__bf16>(ws, h.wc3),
                                                    (long long)P.c2 * bf3_ld(h.kp), bf3_ld(h.kp), P.c2,
                                                    at<float>(ws, h.bc), h.relu_from, at<float>(ws, P.feats[h.out].y),
                                                    P.c2, c->training ? at<float>(ws, h.part) : nullptr, s,
                                                    h.id ? &ida : nullptr, bnf, gfin ? &fbn : nullptr));
        else
            TL(HGNN_K_GEMM_FWD, launch_gemm3_fwd(at<float>(ws, h.a), h.kp, tot, cap, h.kp, at<float>(ws, h.wc), h.kp,
                                                 P.c2, at<float>(ws, h.bc), h.relu_from,
                                                 at<float>(ws, P.feats[h.out].y), P.c2,
                                                 c->training ? at<float>(ws, h.part) : nullptr, s, lg ? 1 : 0));

        BnFwdArgs bf{};
        bf.acc = bnf;
        bf.part = at<float>(ws, h.part);
        bf.tiles = gemm_fwd_tiles_m(cap);
        bf.c = P.c2;
        bf.count = tot;
        bf.w = prm[h.pbn_w];
        bf.b = prm[h.pbn_b];
        bf.mean = at<float>(ws, h.mean);
        bf.std = at<float>(ws, h.stdv);
        bf.run_mean = run ? run[2 * h.bn] : nullptr;
        bf.run_std = run ? run[2 * h.bn + 1] : nullptr;
        bf.training = c->training;
        bf.momentum = 0.1f;
        if (!c->training && !run) return HGNN_ERR_ARG;
        if (!gfin) TL(HGNN_K_BN_FWD, launch_bn_finalize(bf, s));
    }

    AggFwdArgs ag{};
    ag.total_rows = tot_n;
    ag.cap_rows = P.cap_n;
    ag.g = src.v[S_W];
    ag.xg = feat_src(P, ws, P.last_gin, src.x0, src.xl0);
    ag.gbn = feat_bn(P, ws, prm, P.last_gin);
    ag.cg = P.feats[P.last_gin].c;
    ag.jtot = P.jt;
    if (P.last_pin >= 0) {
        ag.p = src.v[S_PN];
        ag.xp = feat_src(P, ws, P.last_pin, src.x0, src.xl0);
        ag.pbn = feat_bn(P, ws, prm, P.last_pin);
        ag.cp = P.feats[P.last_pin].c;
    }
    ag.out = at<float>(ws, P.a_last);
    ag.ldo = P.k_last;
    TL(HGNN_K_AGG_FWD, launch_agg_fwd(ag, s));
    TL(HGNN_K_READOUT, launch_readout_fwd(at<float>(ws, P.a_last), P.k_last, m.node_off, c->bs, c->nmax, prm[P.p_fcw],
                           prm[P.p_fcb], c->dim_out, at<float>(ws, P.colsum), out, s));
    return 0;
}

int net_backward(const hgnn_net_config* c, const hgnn_net_inputs* in, const hgnn_csr_batch* csr,
                 const float* const* prm, void* ws, const float* dout, float* const* grads, float* dX, float* dW,
                 hipStream_t s, Timer* tm, void* const* ev = nullptr, int n_ev = 0) {
    const Program& P = program_of(c);
    if (!fits_32bit(P)) return HGNN_ERR_UNSUPPORTED;
    const Src src = make_src(P, ws, csr);
    BatchMeta m = src.m;
    const int* tot_n = m.totals;
    const int* tot_e = m.totals + 1;
    std::vector<char> init(P.feats.size(), 0);
    auto needs_grad = [&](int f) {
        if (f < 0) return false;
        if (f == 0) return c->need_dx != 0;
        if (c->kind == 1 && f == 1) return false;  // XL never requires grad (scripts/train_mnb.py:56-66)
        return true;
    };
    const bool need_dw = c->need_dw != 0;
    if (need_dw && (!dW || !in || !in->d_X || csr)) return HGNN_ERR_ARG;
    // dense dW contribution of one graph_oper(W, X_l): G block of dA (node rows) x X_l
    auto dw_args = [&](int gin, const float* da, int lda, bool readout, int accumulate) -> DwDenseArgs {
        DwDenseArgs a{};
        a.dA = da;
        a.lda = lda;
        a.f = P.feats[gin].c;
        a.jt = P.jt;
        if (gin == 0) {
            a.xdense = in->d_X;
        } else {
            a.xp = feat_src(P, ws, gin, src.x0, src.xl0);
            const BnView v = feat_bn(P, ws, prm, gin);
            a.pmean = v.mean;
            a.pstd = v.std;
            a.pw = v.w;
            a.pb = v.b;
        }
        if (readout) {
            a.dout = dout;
            a.fcw = prm[P.p_fcw];
            a.dim_out = c->dim_out;
            a.kfc = P.k_last;
        }
        a.node_off = m.node_off;
        a.bs = c->bs;
        a.nmax = c->nmax;
        a.dW = dW;
        a.accumulate = accumulate;
        return a;
    };
    auto dw_dense = [&](int gin, const float* da, int lda, bool readout, int accumulate) -> int {
        return launch_dw_dense(dw_args(gin, da, lda, readout, accumulate), s);
    };

    SideStream* side = nullptr;
    // HGNN_SIDE=0: the weight-gradient work stays on the main stream, with no events at all (a
    // cross-stream event record / wait costs the main stream ~6-7 us of idle GPU per fork)
    static const bool use_side = env_flag("HGNN_SIDE", true);
    if (use_side) TRY(side_stream(s, &side));
    static const bool serial_bwd = env_flag("HGNN_SERIAL_BWD", false);
    // the readout's parameter gradients and its dense dW only feed gradients: on the side stream, forked
    // here, beside the main stream's readout aggregation backward and first halves
    hipStream_t rs = s;
    if (side && !serial_bwd) {
        HGNN_HOST_CHECK(hipEventRecord(side->fork[1], s));
        HGNN_HOST_CHECK(hipStreamWaitEvent(side->s, side->fork[1], 0));
        rs = side->s;
    }
    // readout
    {
        hipStream_t main_s = s;
        s = rs;  // TL records its timer events on the stream the kernel runs on
        TL(HGNN_K_READOUT, launch_readout_bwd_params(dout, at<float>(ws, P.colsum), c->bs, c->nmax, c->dim_out,
                                                     P.k_last, grads[P.p_fcw], grads[P.p_fcb],
                                                     at<void>(ws, P.rb_scratch), s));
        s = main_s;
    }
    // HGNN_READOUT_ROW=0: the readout gradient materialised as a [rows][K] buffer and gathered.  The
    // readout-row kernels hold a graph's rows in LDS: configurations beyond it (wide 2d with a large
    // Nmax / Emax) take the materialised form as well.
    static const bool ro_row = env_flag("HGNN_READOUT_ROW", true);
    const bool lgr = needs_grad(P.last_gin), lpr = needs_grad(P.last_pin);
    ReadoutAggArgs ra{};
    ra.dout = dout;
    ra.fcw = prm[P.p_fcw];
    ra.dim_out = c->dim_out;
    ra.k = P.k_last;
    ra.jt = P.jt;
    ra.cg = P.feats[P.last_gin].c;
    ra.cp = P.last_pin >= 0 ? P.feats[P.last_pin].c : 0;
    ra.bs = c->bs;
    ra.node_off = m.node_off;
    ra.edge_off = m.edge_off;
    ra.g = src.v[S_WT];
    ra.g_total = tot_n;
    ra.g_cap = P.cap_n;
    ra.g_out = lgr ? at<float>(ws, P.feats[P.last_gin].grad) : nullptr;
    ra.g_acc = init[P.last_gin];
    if (lpr) {
        ra.p = src.v[S_PE];
        ra.p_total = tot_e;
        ra.p_cap = P.cap_e;
        ra.p_out = at<float>(ws, P.feats[P.last_pin].grad);
        ra.p_acc = init[P.last_pin];
    }
    const DwDenseArgs dwr = need_dw ? dw_args(P.last_gin, nullptr, 0, true, 0) : DwDenseArgs{};
    if (ro_row && (lgr || lpr || need_dw) && readout_row_fits(ra, need_dw ? &dwr : nullptr)) {
        if (need_dw) {
            hipStream_t main_s = s;
            s = rs;
            TL(HGNN_K_DW_DENSE, launch_dw_readout(dwr, s));
            s = main_s;
        }
        // the readout class (k_readout_agg_bwd: R_b broadcast, no dA read), not agg_bwd: the aggregation
        // class and its HBM roofline are the k_agg_bwd gathers of the halves
        if (lgr || lpr) TL(HGNN_K_READOUT, launch_readout_agg_bwd(ra, s));
        if (lgr) init[P.last_gin] = 1;
        if (lpr) init[P.last_pin] = 1;
    } else if (needs_grad(P.last_gin) || needs_grad(P.last_pin) || need_dw) {
        float* da = at<float>(ws, P.da);
        TL(HGNN_K_READOUT, launch_readout_bwd_da(dout, m.node_off, c->bs, P.cap_n, tot_n, prm[P.p_fcw], c->dim_out, P.k_last,
                                  da, s));
        if (need_dw) TL(HGNN_K_DW_DENSE, dw_dense(P.last_gin, da, P.k_last, true, 0));
        const int cg = P.feats[P.last_gin].c;
        const bool lg = needs_grad(P.last_gin), lp = needs_grad(P.last_pin);
        AggBwdArgs gab{}, pab{};
        if (lg) {
            gab.total_rows = tot_n;
            gab.cap_rows = P.cap_n;
            gab.g = src.v[S_WT];
            gab.ing = da;
            gab.ldg = P.k_last;
            gab.gofs = 0;
            gab.jtot = P.jt;
            gab.c = cg;
            gab.out = at<float>(ws, P.feats[P.last_gin].grad);
            gab.ldo = cg;
            gab.accumulate = init[P.last_gin];
        }
        if (lp) {
            const int cp = P.feats[P.last_pin].c;
            pab.total_rows = tot_e;
            pab.cap_rows = P.cap_e;
            pab.p = src.v[S_PE];
            pab.inp = da;
            pab.ldp = P.k_last;
            pab.pofs_m = P.jt * cg;
            pab.pofs_d = P.jt * cg + cp;
            pab.jtot = P.jt;
            pab.c = cp;
            pab.out = at<float>(ws, P.feats[P.last_pin].grad);
            pab.ldo = cp;
            pab.accumulate = init[P.last_pin];
        }
        if (lg && lp) TL(HGNN_K_AGG_BWD, launch_agg_bwd_pair(gab, pab, s));
        else if (lg) TL(HGNN_K_AGG_BWD, launch_agg_bwd(gab, s));
        else if (lp) TL(HGNN_K_AGG_BWD, launch_agg_bwd(pab, s));
        if (lg) init[P.last_gin] = 1;
        if (lp) init[P.last_pin] = 1;
    }

    // dY, the bias partials and the side-read dA of the q-th half (of the reverse walk) live in ring slot
    // q % nbuf, so the side stream's dW of an earlier half may still read its slot while the main stream runs
    // the next halves; the main stream waits for the side stream only where a slot comes round again (more
    // than BWD_NBUF halves) and once at the end.  (Two alternating slots and a join per half before round 4:
    // each mid-backward join idles the main stream.)
    bool pending[BWD_NBUF] = {};
    int slot = 0, q = 0;
    // the walk leaves region H % 2 zeroed; with an odd number of halves region 0 is not, so a second backward of
    // the same forward (retain_graph) would meet the first one's sums: zeroed here
    if (bn_acc_on() && P.halves.size() % 2 == 1)
        HGNN_HOST_CHECK(hipMemsetAsync(at<double>(ws, P.bnb_acc[0]), 0, (size_t)bn_acc_doubles(P.c2) * sizeof(double), s));
    // HGNN_BWD_TAIL=0: the round-4 tail (the last half forks after its dA GEMM, dX unpacked after the join)
    static const bool bwd_tail = env_flag("HGNN_BWD_TAIL", true);
    // The side stream also takes the dense operator gradient (W.requires_grad) of a node
    // half: it only accumulates into dW, so it leaves the dA -> aggregation-backward chain.
    // (Measured alternative, not kept: the gather half of the aggregation backward on a third
    // stream, overlapping the next half -- 268K vs 286K graphs/s: the concurrent memory-bound
    // kernels only slowed each other.)
    auto fork_dw = [&](const Half& h, int cap, const int* tot, float* dyb, float* dbp, bool ndw_side,
                       float* dab) -> int {
        const int nz = dw3_chunks(cap, P.c2, h.k);
        if (side) {
            HGNN_HOST_CHECK(hipEventRecord(side->fork[q & 1], s));
            HGNN_HOST_CHECK(hipStreamWaitEvent(side->s, side->fork[q & 1], 0));
        }
        hipStream_t main_s = s;
        // HGNN_SERIAL_BWD=1 (diagnostics): everything on the main stream, so a kernel trace shows
        // each kernel's standalone duration
        static const bool serial = env_flag("HGNN_SERIAL_BWD", false);
        if (side && !serial) s = side->s;  // TL records its timer events on the stream the kernel runs on
        int r = 0;
        do {
            if (ndw_side) TL(HGNN_K_DW_DENSE, dw_dense(h.gin, dab, h.kp, false, 1));
            // dY rows have stride c2p; the dW GEMM's float4 loads along the 2d outputs read the zero
            // padding of an odd 2d and store only the 2d real rows of each slab
            const DiagIdArgs ida = diag_id_args(P, ws, prm, h);
            TL(HGNN_K_GEMM_DW, launch_gemm3_dw(dyb, P.c2p, at<float>(ws, h.a), h.kpa, tot, cap, P.c2, h.k, nz,
                                               at<float>(ws, P.slabs), s, h.id ? &ida : nullptr));
            TL(HGNN_K_DW_REDUCE, launch_dw_reduce2(at<float>(ws, P.slabs), tot, nz, P.c2, P.c2, h.k, P.d,
                                                   grads[h.pw_lin], grads[h.pw_relu], dbp, grads[h.pb_lin],
                                                   grads[h.pb_relu], s));
            // a join only where the slot comes round again (the end of the backward has its own)
            if (side && q + P.nbuf < (int)P.halves.size())
                r = hipEventRecord(side->join[slot], s) == hipSuccess ? 0 : HGNN_ERR_HIP;
        } while (0);
        s = main_s;
        pending[slot] = side != nullptr && q + P.nbuf < (int)P.halves.size();
        return r;
    };
    // per-layer completion events (hgnn_net_backward_ex): recorded once the first half (in program
    // order) of a layer -- the last one the reverse walk reaches -- has been enqueued
    const bool lgk = c->kind == 1;
    auto mark = [&](int hd) -> int {
        if (!ev || n_ev <= 0 || (lgk && hd % 2 != 0)) return 0;
        const int l = lgk ? hd / 2 : hd;
        if (2 * l + 1 >= n_ev) return 0;
        HGNN_HOST_CHECK(hipEventRecord(static_cast<hipEvent_t>(ev[2 * l]), s));
        HGNN_HOST_CHECK(hipEventRecord(static_cast<hipEvent_t>(ev[2 * l + 1]), side ? side->s : s));
        return 0;
    };
    auto half_bwd = [&](int hi) -> int {
        const Half& h = P.halves[hi];
        const int cap = h.edge ? P.cap_e : P.cap_n;
        const int* tot = h.edge ? tot_e : tot_n;
        float* dyb = at<float>(ws, P.dyk[slot]);
        float* dbp = at<float>(ws, P.dbk[slot]);
        if (pending[slot]) {  // the dW nbuf halves back still reads this slot
            HGNN_HOST_CHECK(hipStreamWaitEvent(s, side->join[slot], 0));
            pending[slot] = false;
        }
        if (!init[h.out]) HGNN_HOST_CHECK(hipMemsetAsync(at<float>(ws, P.feats[h.out].grad), 0,
                                                          (size_t)cap * P.c2 * sizeof(float), s));
        BnBwdArgs bb{};
        bb.y = at<float>(ws, P.feats[h.out].y);
        bb.dz = at<float>(ws, P.feats[h.out].grad);
        bb.total_rows = tot;
        bb.cap_rows = cap;
        bb.c = P.c2;
        bb.mean = at<float>(ws, h.mean);
        bb.std = at<float>(ws, h.stdv);
        bb.w = prm[h.pbn_w];
        bb.relu_from = h.relu_from;
        bb.training = c->training;
        bb.part = at<float>(ws, P.bnb_part);
        bb.sums = at<float>(ws, P.bnb_sums);
        bb.dy = dyb;
        bb.dw = grads[h.pbn_w];
        bb.db = grads[h.pbn_b];
        bb.dbpart = dbp;
        bb.ldy = P.c2p;
        if (bn_acc_on()) {  // ping-pong: apply4 of this half zeroes the next half's region
            bb.acc64 = at<double>(ws, P.bnb_acc[q % 2]);
            bb.acc64_zero = at<double>(ws, P.bnb_acc[(q + 1) % 2]);
        }

        const bool ng = needs_grad(h.gin), np = needs_grad(h.pin);
        const bool ndw = need_dw && !h.edge;
        TL(HGNN_K_BN_BWD, launch_bn_backward(bb, s));

        if (!ng && !np && !ndw) {
            TRY(fork_dw(h, cap, tot, dyb, dbp, false, nullptr));
            return 0;
        }
        // the side stream's dense dW reads a node half's dA: its own slot buffer; other halves share P.da
        const bool ndw_side = ndw && side;
        float* da = at<float>(ws, ndw_side && P.dak[slot] ? P.dak[slot] : P.da);
        // the last half of the walk (no dense dW, which reads dA) forks before its dA GEMM: the side stream's
        // dW + reduce is the step's tail there, nothing on the main stream follows to overlap it
        const bool early = side && hi == 0 && !ndw && bwd_tail;
        if (early) TRY(fork_dw(h, cap, tot, dyb, dbp, false, nullptr));
        if (da_bf3(P))
            TL(HGNN_K_GEMM_DA, launch_gemm_bf3_da(dyb, P.c2p, tot, cap, P.c2p, at<__bf16>(ws, h.wt3),
                                                  (long long)h.k * bf3_ld(P.c2p), bf3_ld(P.c2p), h.k, da, h.kp, s));
        else
            TL(HGNN_K_GEMM_DA, launch_gemm3_da(dyb, P.c2p, tot, cap, P.c2p, at<float>(ws, h.wt), P.c2p, h.k, da, h.kp,
                                               s));
        // dW starts once dA is done: two MFMA GEMMs side by side only slow each other,
        // dW beside the latency-bound dense-dW / aggregation-backward kernels does not
        if (!early) TRY(fork_dw(h, cap, tot, dyb, dbp, ndw, da));
        AggBwdArgs gab{}, pab{};
        if (ng) {
            gab.total_rows = tot;
            gab.cap_rows = cap;
            gab.g = src.v[h.edge ? S_WLT : S_WT];
            gab.ing = da;
            gab.ldg = h.kp;
            gab.gofs = 0;
            gab.jtot = P.jt;
            gab.c = h.cg;
            gab.out = at<float>(ws, P.feats[h.gin].grad);
            gab.ldo = h.cg;
            gab.accumulate = init[h.gin];
        }
        if (np) {
            const bool other_edge = !h.edge;
            pab.total_rows = other_edge ? tot_e : tot_n;
            pab.cap_rows = other_edge ? P.cap_e : P.cap_n;
            pab.p = src.v[h.edge ? S_PN : S_PE];
            pab.inp = da;
            pab.ldp = h.kp;
            pab.pofs_m = P.jt * h.cg;
            pab.pofs_d = P.jt * h.cg + h.cp;
            pab.jtot = P.jt;
            pab.c = h.cp;
            pab.out = at<float>(ws, P.feats[h.pin].grad);
            pab.ldo = h.cp;
            pab.accumulate = init[h.pin];
        }
        if (ng && np) TL(HGNN_K_AGG_BWD, launch_agg_bwd_pair(gab, pab, s));
        else if (ng) TL(HGNN_K_AGG_BWD, launch_agg_bwd(gab, s));
        else if (np) TL(HGNN_K_AGG_BWD, launch_agg_bwd(pab, s));
        if (ng) init[h.gin] = 1;
        if (np) init[h.pin] = 1;
        return 0;
    };
    for (int hi = (int)P.halves.size() - 1; hi >= 0; --hi, ++q, slot = q % P.nbuf) {
        TRY(half_bwd(hi));
        TRY(mark(hi));
    }
    auto join_side = [&]() -> int {  // the side stream runs in order: its last work done means all of it is
        if (side) {
            HGNN_HOST_CHECK(hipEventRecord(side->join[BWD_NBUF], side->s));
            HGNN_HOST_CHECK(hipStreamWaitEvent(s, side->join[BWD_NBUF], 0));
        }
        return 0;
    };
    // dX reads only the main stream's aggregation gradients: unpacked before the join (HGNN_BWD_TAIL=0: after)
    if (!bwd_tail) TRY(join_side());
    if (c->need_dx) {
        if (!dX) return HGNN_ERR_ARG;
        if (!init[0]) HGNN_HOST_CHECK(hipMemsetAsync(at<float>(ws, P.feats[0].grad), 0,
                                                     (size_t)P.cap_n * c->f_in * sizeof(float), s));
        if (csr)
            HGNN_HOST_CHECK(hipMemcpyAsync(dX, at<float>(ws, P.feats[0].grad), (size_t)src.nodes * c->f_in * sizeof(float),
                                           hipMemcpyDeviceToDevice, s));
        else
            TL(HGNN_K_STRUCT, launch_unpack_nodes(at<float>(ws, P.feats[0].grad), c->bs, c->f_in, c->nmax, m, dX, s));
    }
    if (bwd_tail) TRY(join_side());
    return 0;
}

// ---- Replay of launch-bound calls.  A small network (config 1: 19 GNN_simple layers over 32 SBM-50 graphs)
// enqueues ~200 kernels of 3-10 us each per step, and the host's enqueue (~2 ms) is the step.  Such a call,
// met a third time with the same configuration and the same device pointers (a training loop: the same input
// tensors, the caching allocator's same workspace / output / gradient blocks), is captured once on a private
// stream into a HIP graph and from then on replayed with one hipGraphLaunch on the caller's stream.  The
// enqueue reads nothing from the host but the configuration and the pointers (no host synchronisation, no
// data-dependent launch), so the replay runs the same kernels on the same buffers.  Not for the headline
// shapes: their kernels outlast the enqueue, and a replayed graph runs the side stream's branch serially
// (DESIGN.md §8 round 3).  HGNN_EXEC_GRAPH=0 never, =1 always, unset: calls of <= 4096 node rows.  Calls
// inside a caller's capture, timed calls and calls with per-layer DP events enqueue as before.
struct ReplayEntry {
    std::vector<uintptr_t> key;
    int seen = 0;
    bool failed = false;
    hipGraphExec_t exec = nullptr;
    hipEvent_t done = nullptr;  // recorded on the caller's stream after each launch of exec
    unsigned long long last = 0;
};

// Destroy an entry's executable graph once its last launch has finished: a wait on that launch's
// event, not a device-wide synchronisation (which would also wait for other streams, e.g. the DP
// communication stream, and is not allowed while another stream of the device is capturing).
static void replay_release(ReplayEntry& x) {
    if (x.done) (void)hipEventSynchronize(x.done);
    if (x.exec) (void)hipGraphExecDestroy(x.exec);
    if (x.done) (void)hipEventDestroy(x.done);
    x.exec = nullptr;
    x.done = nullptr;
}

static int replay_launch(ReplayEntry& x, hipStream_t s) {
    if (hipGraphLaunch(x.exec, s) != hipSuccess) return HGNN_ERR_HIP;
    return hipEventRecord(x.done, s) == hipSuccess ? 0 : HGNN_ERR_HIP;
}
struct ReplayCache {
    std::vector<ReplayEntry> e;
    unsigned long long tick = 0;
    int dev = -1;
    hipStream_t cap = nullptr;
};
constexpr size_t REPLAY_MAX = 16;

static bool replay_eligible(const hgnn_net_config* c) {
    static const int mode = [] {
        const char* v = getenv("HGNN_EXEC_GRAPH");
        return !v ? -1 : (v[0] == '1' ? 1 : (v[0] == '0' ? 0 : -1));
    }();
    if (mode >= 0) return mode == 1;
    return (long long)c->bs * c->nmax <= 4096 && (c->kind == 0 || (long long)c->bs * c->emax <= 8192);
}

struct KeyBuilder {
    std::vector<uintptr_t> k;
    void add(uintptr_t v) { k.push_back(v); }
    void ptr(const void* p) { k.push_back(reinterpret_cast<uintptr_t>(p)); }
    void cfg(const hgnn_net_config* c) {
        const int32_t* w = reinterpret_cast<const int32_t*>(c);
        for (size_t i = 0; i < sizeof(hgnn_net_config) / 4; ++i) add((uintptr_t)(uint32_t)w[i]);
    }
    void inputs(const hgnn_net_inputs* in) {
        if (!in) return add(0);
        const void* const* p = reinterpret_cast<const void* const*>(in);
        for (size_t i = 0; i < sizeof(hgnn_net_inputs) / sizeof(void*); ++i) ptr(p[i]);
    }
    void csr(const hgnn_csr_batch* b) {
        if (!b) return add(0);
        ptr(b->d_node_off);
        ptr(b->d_edge_off);
        ptr(b->d_totals);
        ptr(b->d_n_batch);
        ptr(b->d_e_batch);
        ptr(b->d_x);
        ptr(b->d_xl);
        for (int k = 0; k < S_COUNT; ++k) {
            ptr(b->d_rows[k]);
            ptr(b->d_entries[k]);
        }
        add((uintptr_t)b->stride_w);
        add((uintptr_t)b->nodes);
        add((uintptr_t)b->edges);
    }
    template <typename T>
    void ptrs(T* const* p, int n) {
        for (int i = 0; i < n; ++i) ptr(p ? p[i] : nullptr);
    }
};

static int replay_reset(ReplayCache& rc, int dev) {
    if (rc.dev >= 0) {
        for (auto& x : rc.e) replay_release(x);
        if (rc.cap) (void)hipStreamDestroy(rc.cap);
    }
    rc = ReplayCache{};
    int cur = 0;
    HGNN_HOST_CHECK(hipGetDevice(&cur));
    HGNN_HOST_CHECK(hipSetDevice(dev));
    const hipError_t e = hipStreamCreateWithFlags(&rc.cap, hipStreamNonBlocking);
    HGNN_HOST_CHECK(hipSetDevice(cur));
    if (e != hipSuccess) return HGNN_ERR_HIP;
    rc.dev = dev;
    return 0;
}

template <typename F>
static int replayed(std::vector<uintptr_t> key, hipStream_t s, F&& enqueue) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    HGNN_HOST_CHECK(hipStreamIsCapturing(s, &st));
    if (st != hipStreamCaptureStatusNone) return enqueue(s);  // inside the caller's own capture
    thread_local ReplayCache rc;
    hipDevice_t dev = 0;
    HGNN_HOST_CHECK(hipStreamGetDevice(s, &dev));
    if (rc.dev != dev) TRY(replay_reset(rc, dev));
    ReplayEntry* hit = nullptr;
    for (auto& x : rc.e)
        if (x.key == key) {
            hit = &x;
            break;
        }
    if (hit && hit->exec) {
        hit->last = ++rc.tick;
        return replay_launch(*hit, s);
    }
    if (!hit) {
        if (rc.e.size() >= REPLAY_MAX) {  // evict the least recently used entry
            size_t v = 0;
            for (size_t i = 1; i < rc.e.size(); ++i)
                if (rc.e[i].last < rc.e[v].last) v = i;
            replay_release(rc.e[v]);  // waits for its last launch only
            rc.e.erase(rc.e.begin() + v);
        }
        rc.e.push_back(ReplayEntry{});
        hit = &rc.e.back();
        hit->key = std::move(key);
    }
    hit->last = ++rc.tick;
    if (hit->failed || ++hit->seen < 3) return enqueue(s);
    // third call: capture the enqueue on the private stream, replay it on the caller's
    HGNN_HOST_CHECK(hipStreamBeginCapture(rc.cap, hipStreamCaptureModeRelaxed));
    const int r = enqueue(rc.cap);
    hipGraph_t gr = nullptr;
    const hipError_t ee = hipStreamEndCapture(rc.cap, &gr);
    hipGraphExec_t x = nullptr;
    hipEvent_t done = nullptr;
    const bool ok = r == 0 && ee == hipSuccess && gr && hipGraphInstantiate(&x, gr, nullptr, nullptr, 0) == hipSuccess &&
                    hipEventCreateWithFlags(&done, hipEventDisableTiming) == hipSuccess;
    if (gr) (void)hipGraphDestroy(gr);
    if (!ok) {
        (void)hipGetLastError();
        if (x) (void)hipGraphExecDestroy(x);
        hit->failed = true;
        return r ? r : enqueue(s);
    }
    hit->exec = x;
    hit->done = done;
    return replay_launch(*hit, s);
}

static int n_running(const hgnn_net_config* c) { return 2 * (c->kind == 1 ? 2 : 1) * (c->n_layers - 1); }
static int n_params(const hgnn_net_config* c) { return (c->kind == 1 ? 12 : 6) * (c->n_layers - 1) + 2; }

static int forward_call(const hgnn_net_config* c, const hgnn_net_inputs* in, const hgnn_csr_batch* csr,
                        const float* const* prm, float* const* run, void* ws, float* out, hipStream_t s) {
    if (!replay_eligible(c)) return net_forward(c, in, csr, prm, run, ws, out, s, nullptr);
    KeyBuilder k;
    k.add('F');
    k.cfg(c);
    k.inputs(in);
    k.csr(csr);
    k.ptrs(prm, n_params(c));
    k.ptrs(run, n_running(c));
    k.ptr(ws);
    k.ptr(out);
    return replayed(std::move(k.k), s,
                    [&](hipStream_t st) { return net_forward(c, in, csr, prm, run, ws, out, st, nullptr); });
}

static int backward_call(const hgnn_net_config* c, const hgnn_net_inputs* in, const hgnn_csr_batch* csr,
                         const float* const* prm, void* ws, const float* dout, float* const* grads, float* dX,
                         float* dW, hipStream_t s) {
    if (!replay_eligible(c)) return net_backward(c, in, csr, prm, ws, dout, grads, dX, dW, s, nullptr);
    KeyBuilder k;
    k.add('B');
    k.cfg(c);
    k.inputs(in);
    k.csr(csr);
    k.ptrs(prm, n_params(c));
    k.ptr(ws);
    k.ptr(dout);
    k.ptrs(grads, n_params(c));
    k.ptr(dX);
    k.ptr(dW);
    return replayed(std::move(k.k), s, [&](hipStream_t st) {
        return net_backward(c, in, csr, prm, ws, dout, grads, dX, dW, st, nullptr);
    });
}

}  // namespace
}  // namespace hgnn

using namespace hgnn;

extern "C" {

int hgnn_abi_version(void) { return HGNN_ABI_VERSION; }

const char* hgnn_status_string(int status) {
    switch (status) {
        case HGNN_OK: return "ok";
        case HGNN_ERR_ARG: return "invalid argument";
        case HGNN_ERR_UNSUPPORTED: return "unsupported configuration";
        case HGNN_ERR_HIP: return "HIP runtime error";
        case HGNN_ERR_INDEX: return "index out of range";
        default: return "unknown status";
    }
}

int hgnn_net_param_count(const hgnn_net_config* cfg) {
    if (!valid_config(cfg)) return -1;
    return (cfg->kind == 1 ? 12 : 6) * (cfg->n_layers - 1) + 2;
}

int hgnn_net_bn_count(const hgnn_net_config* cfg) {
    if (!valid_config(cfg)) return -1;
    return (cfg->kind == 1 ? 2 : 1) * (cfg->n_layers - 1);
}

size_t hgnn_net_workspace_bytes(const hgnn_net_config* cfg) {
    if (!valid_config(cfg)) return 0;
    const Program& P = program_of(cfg);
    return fits_32bit(P) ? P.bytes : 0;
}

uint32_t* hgnn_net_error_word(const hgnn_net_config* cfg, void* workspace) {
    if (!valid_config(cfg) || !workspace) return nullptr;
    return at<uint32_t>(workspace, program_of(cfg).err);
}

int hgnn_net_forward(const hgnn_net_config* cfg, const hgnn_net_inputs* in, const float* const* params,
                     float* const* bn_running, void* workspace, float* d_out, void* stream) {
    if (!valid_config(cfg) || !in || !params || !workspace || !d_out) return HGNN_ERR_ARG;
    if (!in->d_X || !in->d_W || !in->d_N_batch || !in->d_mask) return HGNN_ERR_ARG;
    if (cfg->kind == 1 && (!in->d_XL || !in->d_WL || !in->d_Pm || !in->d_Pd || !in->d_E_batch || !in->d_mask_lg))
        return HGNN_ERR_ARG;
    return forward_call(cfg, in, nullptr, params, bn_running, workspace, d_out, static_cast<hipStream_t>(stream));
}

int hgnn_net_backward(const hgnn_net_config* cfg, const hgnn_net_inputs* in, const float* const* params,
                      void* workspace, const float* d_dout, float* const* grads, float* d_dX, float* d_dW,
                      void* stream) {
    if (!valid_config(cfg) || !params || !workspace || !d_dout || !grads) return HGNN_ERR_ARG;
    return backward_call(cfg, in, nullptr, params, workspace, d_dout, grads, d_dX, d_dW,
                         static_cast<hipStream_t>(stream));
}

void* hgnn_timer_create_ex(int max_launches, unsigned class_mask, int mode, long long stamp_words) {
    if (max_launches <= 0) return nullptr;
    if (mode != HGNN_TIMER_STAMPS && mode != HGNN_TIMER_DISPATCH && mode != HGNN_TIMER_MARKERS) return nullptr;
    Timer* t = new Timer();
    t->cls.resize(max_launches);
    t->mask = class_mask;
    t->mode = mode;
    if (mode == HGNN_TIMER_STAMPS) {
        if (stamp_words <= 0 || stamp_words > (1ll << 31) - 1) {
            delete t;
            return nullptr;
        }
        t->st_off.resize(max_launches);
        t->st_n.resize(max_launches);
        t->st_strm.resize(max_launches);
        t->st_cap = stamp_words;
        if (hipMalloc(&t->st, (size_t)stamp_words * 8) != hipSuccess ||
            hipMemset(t->st, 0, (size_t)stamp_words * 8) != hipSuccess) {
            if (t->st) (void)hipFree(t->st);
            delete t;
            return nullptr;
        }
        return t;
    }
    t->ev.resize(2 * (size_t)max_launches);
    for (auto& e : t->ev) {
        if (hipEventCreate(&e) != hipSuccess) {
            delete t;
            return nullptr;
        }
    }
    return t;
}

void* hgnn_timer_create(int max_launches, unsigned class_mask) {
    const char* e = getenv("HGNN_TIMER_MARKERS");
    return hgnn_timer_create_ex(max_launches, class_mask,
                                e && e[0] == '1' ? HGNN_TIMER_MARKERS : HGNN_TIMER_DISPATCH, 0);
}

void hgnn_timer_reset(void* timer) {
    if (!timer) return;
    Timer* t = static_cast<Timer*>(timer);
    t->used = 0;
    if (t->st) {
        (void)hipDeviceSynchronize();
        (void)hipMemset(t->st, 0, (size_t)t->st_used * 8);
        t->st_used = 0;
        t->st_read = false;
    }
}

// Stamp mode: a launch's time = max over its waves' exit stamps - min over their entry stamps (100 MHz).
static int timer_read_stamps(Timer* t) {
    if (t->st_read && t->rd_used == t->used && t->rd_st_used == t->st_used) return HGNN_OK;
    if (hipDeviceSynchronize() != hipSuccess) return HGNN_ERR_HIP;
    std::vector<uint64_t> h((size_t)t->st_used);
    if (t->st_used && hipMemcpy(h.data(), t->st, (size_t)t->st_used * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return HGNN_ERR_HIP;
    t->st_ms.assign(t->used, 0.0);
    t->st_lo.assign(t->used, 0);
    t->st_hi.assign(t->used, 0);
    for (int i = 0; i < t->used; ++i) {
        uint64_t lo = ~0ull, hi = 0;
        for (int w = 0; w < t->st_n[i] / 2; ++w) {
            const uint64_t a = h[t->st_off[i] + 2 * w], b = h[t->st_off[i] + 2 * w + 1];
            if (a && a < lo) lo = a;
            if (b > hi) hi = b;
        }
        t->st_ms[i] = hi > lo && lo != ~0ull ? (double)(hi - lo) * 1e-5 : 0.0;  // 10 ns ticks -> ms
        t->st_lo[i] = lo == ~0ull ? 0 : lo;
        t->st_hi[i] = hi;
    }
    t->st_read = true;
    t->rd_used = t->used;
    t->rd_st_used = t->st_used;
    return HGNN_OK;
}

int hgnn_timer_elapsed(void* timer, int kernel_class, double* total_ms, int* launches) {
    if (!timer || !total_ms || !launches) return HGNN_ERR_ARG;
    Timer* t = static_cast<Timer*>(timer);
    double tot = 0.0;
    int n = 0;
    if (t->mode == HGNN_TIMER_STAMPS) {
        const int r = timer_read_stamps(t);
        if (r) return r;
        for (int i = 0; i < t->used; ++i)
            if (t->cls[i] == kernel_class) {
                tot += t->st_ms[i];
                ++n;
            }
        *total_ms = tot;
        *launches = n;
        return HGNN_OK;
    }
    for (int i = 0; i < t->used; ++i) {
        if (t->cls[i] != kernel_class) continue;
        float ms = 0.f;
        if (hipEventSynchronize(t->ev[2 * i + 1]) != hipSuccess) return HGNN_ERR_HIP;
        if (hipEventElapsedTime(&ms, t->ev[2 * i], t->ev[2 * i + 1]) != hipSuccess) return HGNN_ERR_HIP;
        tot += ms;
        ++n;
    }
    *total_ms = tot;
    *launches = n;
    return HGNN_OK;
}

int hgnn_timer_launches(void* timer, int max, int* cls, double* t_entry_us, double* t_exit_us, int* stream_idx) {
    if (!timer || max < 0 || (max > 0 && (!cls || !t_entry_us || !t_exit_us))) return -HGNN_ERR_ARG;
    Timer* t = static_cast<Timer*>(timer);
    if (t->mode != HGNN_TIMER_STAMPS) return -HGNN_ERR_UNSUPPORTED;
    const int r = timer_read_stamps(t);
    if (r) return -r;
    uint64_t base = ~0ull;
    for (int i = 0; i < t->used; ++i)
        if (t->st_lo[i] && t->st_lo[i] < base) base = t->st_lo[i];
    const int n = t->used < max ? t->used : max;
    std::vector<uintptr_t> seen;
    for (int i = 0; i < n; ++i) {
        cls[i] = t->cls[i];
        if (stream_idx) {
            int q = 0;
            while (q < (int)seen.size() && seen[q] != t->st_strm[i]) ++q;
            if (q == (int)seen.size()) seen.push_back(t->st_strm[i]);
            stream_idx[i] = q;
        }
        t_entry_us[i] = t->st_lo[i] ? (double)(t->st_lo[i] - base) * 1e-2 : -1.0;
        t_exit_us[i] = t->st_hi[i] ? (double)(t->st_hi[i] - base) * 1e-2 : -1.0;
    }
    return t->used;
}

long long hgnn_timer_waves(void* timer, int launch, long long max, double* entry_us, double* exit_us) {
    if (!timer || max < 0 || (max > 0 && (!entry_us || !exit_us))) return -HGNN_ERR_ARG;
    Timer* t = static_cast<Timer*>(timer);
    if (t->mode != HGNN_TIMER_STAMPS) return -HGNN_ERR_UNSUPPORTED;
    if (launch < 0 || launch >= t->used) return -HGNN_ERR_ARG;
    if (hipDeviceSynchronize() != hipSuccess) return -HGNN_ERR_HIP;
    const int r = timer_read_stamps(t);
    if (r) return -r;
    uint64_t base = ~0ull;
    for (int i = 0; i < t->used; ++i)
        if (t->st_lo[i] && t->st_lo[i] < base) base = t->st_lo[i];
    const long long nw = t->st_n[launch] / 2, n = nw < max ? nw : max;
    if (n > 0) {
        std::vector<uint64_t> h((size_t)(2 * n));
        if (hipMemcpy(h.data(), t->st + t->st_off[launch], (size_t)(2 * n) * 8, hipMemcpyDeviceToHost) != hipSuccess)
            return -HGNN_ERR_HIP;
        for (long long w = 0; w < n; ++w) {
            entry_us[w] = h[2 * w] ? (double)(h[2 * w] - base) * 1e-2 : -1.0;
            exit_us[w] = h[2 * w + 1] ? (double)(h[2 * w + 1] - base) * 1e-2 : -1.0;
        }
    }
    return nw;
}

void hgnn_timer_destroy(void* timer) {
    if (!timer) return;
    Timer* t = static_cast<Timer*>(timer);
    for (auto& e : t->ev) (void)hipEventDestroy(e);
    if (t->st) {
        (void)hipDeviceSynchronize();
        (void)hipFree(t->st);
    }
    delete t;
}

int hgnn_net_forward_timed(const hgnn_net_config* cfg, const hgnn_net_inputs* in, const float* const* params,
                           float* const* bn_running, void* workspace, float* d_out, void* stream, void* timer) {
    if (!valid_config(cfg) || !in || !params || !workspace || !d_out) return HGNN_ERR_ARG;
    return net_forward(cfg, in, nullptr, params, bn_running, workspace, d_out, static_cast<hipStream_t>(stream),
                       static_cast<Timer*>(timer));
}

int hgnn_net_backward_timed(const hgnn_net_config* cfg, const hgnn_net_inputs* in, const float* const* params,
                            void* workspace, const float* d_dout, float* const* grads, float* d_dX, float* d_dW,
                            void* stream, void* timer) {
    if (!valid_config(cfg) || !params || !workspace || !d_dout || !grads) return HGNN_ERR_ARG;
    return net_backward(cfg, in, nullptr, params, workspace, d_dout, grads, d_dX, d_dW,
                        static_cast<hipStream_t>(stream), static_cast<Timer*>(timer));
}

static bool csr_matches(const hgnn_net_config* cfg, const hgnn_csr_batch* b) {
    if (!b || !b->d_node_off || !b->d_totals || !b->d_x || !b->d_rows[S_W] || !b->d_rows[S_WT]) return false;
    if (cfg->kind == 1 && (!b->d_xl || !b->d_rows[S_WL] || !b->d_rows[S_WLT] || !b->d_rows[S_PN] || !b->d_rows[S_PE]))
        return false;
    return b->stride_w == (cfg->j_tot <= 3 ? 4 : 8);
}

int hgnn_csr_batch_view(const hgnn_csr_layout* L, const void* d_base, hgnn_csr_batch* out) {
    if (!L || !d_base || !out) return HGNN_ERR_ARG;
    const char* b = static_cast<const char*>(d_base);
    hgnn_csr_batch r{};
    r.d_node_off = b + L->off_node_off;
    r.d_edge_off = b + L->off_edge_off;
    r.d_totals = b + L->off_totals;
    r.d_n_batch = reinterpret_cast<const int64_t*>(b + L->off_n_batch);
    r.d_e_batch = reinterpret_cast<const int64_t*>(b + L->off_e_batch);
    r.d_x = reinterpret_cast<const float*>(b + L->off_x);
    r.d_xl = reinterpret_cast<const float*>(b + L->off_xl);
    for (int k = 0; k < S_COUNT; ++k) {
        r.d_rows[k] = b + L->off_rows[k];
        r.d_entries[k] = reinterpret_cast<const float*>(b + L->off_entries[k]);
    }
    r.stride_w = L->stride_w;
    r.nodes = L->nodes;
    r.edges = L->edges;
    *out = r;
    return HGNN_OK;
}

int hgnn_net_forward_csr(const hgnn_net_config* cfg, const hgnn_csr_batch* batch, const float* const* params,
                         float* const* bn_running, void* workspace, float* d_out, void* stream) {
    if (!valid_config(cfg) || !csr_matches(cfg, batch) || !params || !workspace || !d_out) return HGNN_ERR_ARG;
    return forward_call(cfg, nullptr, batch, params, bn_running, workspace, d_out, static_cast<hipStream_t>(stream));
}

int hgnn_net_backward_ex(const hgnn_net_config* cfg, const hgnn_net_inputs* in, const hgnn_csr_batch* csr,
                         const float* const* params, void* workspace, const float* d_dout, float* const* grads,
                         float* d_dX, float* d_dW, void* stream, void* timer, void* const* events, int n_events) {
    if (!valid_config(cfg) || !params || !workspace || !d_dout || !grads) return HGNN_ERR_ARG;
    if (csr && (!csr_matches(cfg, csr) || cfg->need_dw)) return HGNN_ERR_ARG;
    if (!csr && cfg->need_dw && (!in || !in->d_X)) return HGNN_ERR_ARG;
    if (n_events < 0 || (n_events > 0 && !events)) return HGNN_ERR_ARG;
    if (!timer && n_events == 0)
        return backward_call(cfg, in, csr, params, workspace, d_dout, grads, d_dX, d_dW, static_cast<hipStream_t>(stream));
    return net_backward(cfg, in, csr, params, workspace, d_dout, grads, d_dX, d_dW, static_cast<hipStream_t>(stream),
                        static_cast<Timer*>(timer), events, n_events);
}

int hgnn_net_backward_csr(const hgnn_net_config* cfg, const hgnn_csr_batch* batch, const float* const* params,
                          void* workspace, const float* d_dout, float* const* grads, float* d_dX, void* stream) {
    if (!valid_config(cfg) || !csr_matches(cfg, batch) || !params || !workspace || !d_dout || !grads)
        return HGNN_ERR_ARG;
    if (cfg->need_dw) return HGNN_ERR_ARG;
    return backward_call(cfg, nullptr, batch, params, workspace, d_dout, grads, d_dX, nullptr,
                         static_cast<hipStream_t>(stream));
}

}  // extern "C"
