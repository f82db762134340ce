// capi.cpp -- implementation of include/fa2_amd.h on top of the launch layer
// (namespace fa2, declared in kernels/f-attn2.cuh).
#include "fa2_amd.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

#include "f-attn.cuh"
#include "f-attn2.cuh"
#include "vanilla-attn.cuh"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int check_shape(int B, int H, int S, int D) {
    if (B <= 0 || H <= 0 || S <= 0) return fail(FA2_E_INVALID, "batch, heads and seq must be positive");
    if (!fa2::supported_head_dim(D)) return fail(FA2_E_INVALID, "head_dim must be 32, 64 or 128");
    if ((long long)B * H * S * D > 0x7fffffffLL * 4)
        return fail(FA2_E_INVALID, "tensor too large (B*H*S*D must fit the 32-bit launch grid)");
    if ((long long)B * H > 0x7fffffffLL / ((S + 31) / 32)) return fail(FA2_E_INVALID, "grid too large");
    return FA2_OK;
}

int check_ptrs(std::initializer_list<const void*> ps) {
    for (const void* p : ps)
        if (!p) return fail(FA2_E_INVALID, "null tensor pointer");
    return FA2_OK;
}

int hip_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return FA2_OK;
    return fail(e == hipErrorOutOfMemory ? FA2_E_NOMEM : FA2_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

int check_precision(int precision) {
    if (precision != FA2_FP16 && precision != FA2_FP32 && precision != FA2_BF16)
        return fail(FA2_E_INVALID, "precision must be FA2_FP16, FA2_FP32 or FA2_BF16");
    return FA2_OK;
}

}  // namespace

namespace {
// launch-plan overrides set through fa2_tune_set (empty in production)
std::mutex g_tune_mu;
std::vector<std::pair<std::string, int>> g_tune;
std::atomic<int> g_tune_n{0};

// the launch-plan overrides the launchers read (fa2_tune_set rejects other names,
// so a misspelt knob cannot silently leave an A/B on the default plan)
const char* const kKnobs[] = {"FWD_HS",   "FWD_WAVES", "FWD_KS",          "FWD_NKB", "DKDV_WAVES", "DKDV_QS",
                              "DKDV_HS",  "DQ_WAVES",  "DQ_KS",           "DQ_HS",   "BWD_FUSED",  "BWD_FUSED_DELTA",
                              "BWD_FQS",  "BWD_FKS",   "BWD_FNW",         "HOST_SHARDS_ON_DEVICE0",    "HOST_CHUNKS",
                              "FWD_SPLIT", "BWD_SPLIT"};
bool known_knob(const char* k) {
    for (const char* n : kKnobs)
        if (!strcmp(n, k)) return true;
    return false;
}
}  // namespace

namespace fa2 {
int tune_knob(const char* name, int dflt) {
    if (g_tune_n.load(std::memory_order_acquire) == 0) return dflt;
    std::lock_guard<std::mutex> lock(g_tune_mu);
    for (const auto& kv : g_tune)
        if (kv.first == name) return kv.second;
    return dflt;
}

int cu_count() {
    static std::atomic<int> ncu_cache[64] = {};
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64) {
        if (!ncu_cache[dev].load(std::memory_order_relaxed)) {
            int n = 0;
            if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
                ncu_cache[dev].store(n, std::memory_order_relaxed);
        }
        if (const int c = ncu_cache[dev].load(std::memory_order_relaxed)) ncu = c;
    }
    return ncu;
}

// per-(device, stream) scratch of the split plans (f-attn2.cuh: stream_scratch)
struct StreamScratch {
    int device;
    hipStream_t stream;
    void* p;
    size_t bytes;
    unsigned long long capture = 0;  // the capture that took it (graph-owned blocks)
};
std::mutex g_scr_mu;
std::vector<StreamScratch> g_scr;    // eager calls' blocks, one per (device, stream)
std::vector<StreamScratch> g_scr_g;  // blocks handed to graph captures (owned by the graphs)

void* stream_scratch(hipStream_t stream, size_t bytes) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    unsigned long long cap = 0;
    if (hipStreamGetCaptureInfo(stream, &cs, &cap) != hipSuccess) return nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lock(g_scr_mu);
    if (cs != hipStreamCaptureStatusNone) {
        // a capture cannot allocate: it takes the stream's block from an earlier eager call
        // (the usual warm-up before a capture), which then belongs to the graph -- later eager
        // calls get a block of their own, so a replay and eager work never share one.  Later
        // requests of the same capture (the backward after the forward) reuse that block:
        // they are ordered on the capture stream like the eager calls they replay.
        if (cs != hipStreamCaptureStatusActive) return nullptr;
        for (auto& e : g_scr_g)
            if (e.capture == cap && e.device == dev && e.stream == stream) return e.bytes >= bytes ? e.p : nullptr;
        for (size_t i = 0; i < g_scr.size(); ++i)
            if (g_scr[i].device == dev && g_scr[i].stream == stream && g_scr[i].bytes >= bytes) {
                g_scr_g.push_back(g_scr[i]);
                g_scr_g.back().capture = cap;
                g_scr.erase(g_scr.begin() + (long)i);
                return g_scr_g.back().p;
            }
        return nullptr;
    }
    for (auto& e : g_scr) {
        if (e.device != dev || e.stream != stream) continue;
        if (e.bytes >= bytes) return e.p;
        // grow: the stream's earlier launches may still read the old block
        if (hipStreamSynchronize(stream) != hipSuccess) return nullptr;
        (void)hipFree(e.p);
        e.p = nullptr;
        e.bytes = 0;
        if (hipMalloc(&e.p, bytes) != hipSuccess) return e.p = nullptr;
        e.bytes = bytes;
        return e.p;
    }
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    g_scr.push_back({dev, stream, p, bytes});
    return p;
}

void stream_scratch_release() {
    int dev0 = 0;
    const bool have = hipGetDevice(&dev0) == hipSuccess;
    std::lock_guard<std::mutex> lock(g_scr_mu);
    for (auto* v : {&g_scr, &g_scr_g}) {
        for (auto& e : *v) {
            (void)hipSetDevice(e.device);
            (void)hipFree(e.p);
        }
        v->clear();
    }
    if (have) (void)hipSetDevice(dev0);
}

int auto_waves(long blocks32, int maxnw, int minnw) {
    const int ncu = cu_count();
    for (int nw = maxnw; nw > minnw; nw /= 2)
        if ((blocks32 + nw - 1) / nw >= ncu) return nw;
    return minnw;
}
}  // namespace fa2

extern "C" {

int fa2_version(void) { return 2 * 10000 + 1 * 100 + 0; }  // 2.1: split forward, per-stream scratch

#ifndef FA2_BUILD_ID
#define FA2_BUILD_ID "unknown"
#endif
const char* fa2_build_id(void) { return FA2_BUILD_ID; }

int fa2_tune_set(const char* knob, int value) {
    if (knob && !known_knob(knob)) return fail(FA2_E_INVALID, "unknown knob name");
    std::lock_guard<std::mutex> lock(g_tune_mu);
    if (!knob) {
        g_tune.clear();
    } else {
        bool found = false;
        for (auto& kv : g_tune)
            if (kv.first == knob) kv.second = value, found = true;
        if (!found) g_tune.emplace_back(knob, value);
    }
    g_tune_n.store((int)g_tune.size(), std::memory_order_release);
    return FA2_OK;
}

int fa2_tune_get(const char* knob, int* value) {
    if (!knob || !known_knob(knob)) return fail(FA2_E_INVALID, "unknown knob name");
    std::lock_guard<std::mutex> lock(g_tune_mu);
    for (const auto& kv : g_tune)
        if (kv.first == knob) {
            if (value) *value = kv.second;
            return 1;
        }
    return 0;
}

const char* fa2_last_error(void) { return g_err.c_str(); }

int fa2_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int fa2_shard_range(int total_heads, int shards, int index, int* first, int* count) {
    if (total_heads < 0 || shards <= 0 || index < 0 || index >= shards || !first || !count)
        return fail(FA2_E_INVALID, "bad shard arguments");
    const int q = total_heads / shards, r = total_heads % shards;
    *first = index * q + std::min(index, r);
    *count = q + (index < r ? 1 : 0);
    return FA2_OK;
}

int fa2_forward(const float* q, const float* k, const float* v, float* o, float* lse, int B, int H, int S, int D,
                int precision, void* stream) {
    int rc;
    if ((rc = check_shape(B, H, S, D)) || (rc = check_precision(precision)) || (rc = check_ptrs({q, k, v, o, lse})))
        return rc;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const hipError_t e = precision == FA2_FP16   ? fa2::launch_forward_f16(D, q, k, v, o, lse, B * H, S, st)
                         : precision == FA2_BF16 ? fa2::launch_forward_bf16(D, q, k, v, o, lse, B * H, S, st)
                                                 : fa2::launch_forward_f32(D, q, k, v, o, lse, B * H, S, st);
    return hip_status(e, "fa2_forward launch");
}

int fa2_delta(const float* dout, const float* o, float* delta, int B, int H, int S, int D, void* stream) {
    int rc;
    if ((rc = check_shape(B, H, S, D)) || (rc = check_ptrs({dout, o, delta}))) return rc;
    return hip_status(fa2::launch_delta(D, dout, o, delta, B * H, S, static_cast<hipStream_t>(stream)),
                      "fa2_delta launch");
}

int fa2_backward(const float* q, const float* k, const float* v, const float* o, const float* dout, const float* lse,
                 float* delta, float* dq, float* dk, float* dv, int B, int H, int S, int D, int precision,
                 void* stream) {
    int rc;
    if ((rc = check_shape(B, H, S, D)) || (rc = check_precision(precision)) ||
        (rc = check_ptrs({q, k, v, o, dout, lse, delta, dq, dk, dv})))
        return rc;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const hipError_t e =
        precision == FA2_FP16   ? fa2::launch_backward_f16(D, q, k, v, o, dout, lse, delta, dq, dk, dv, B * H, S, st)
        : precision == FA2_BF16 ? fa2::launch_backward_bf16(D, q, k, v, o, dout, lse, delta, dq, dk, dv, B * H, S, st)
                                : fa2::launch_backward_f32(D, q, k, v, o, dout, lse, delta, dq, dk, dv, B * H, S, st);
    return hip_status(e, "fa2_backward launch");
}

int fa2_backward_dkdv(const float* q, const float* k, const float* v, const float* dout, const float* lse,
                      const float* delta, float* dk, float* dv, int B, int H, int S, int D, void* stream) {
    int rc;
    if ((rc = check_shape(B, H, S, D)) || (rc = check_ptrs({q, k, v, dout, lse, delta, dk, dv}))) return rc;
    return hip_status(
        fa2::launch_bwd_dkdv_f16(D, q, k, v, dout, lse, delta, dk, dv, B * H, S, static_cast<hipStream_t>(stream)),
        "fa2_backward_dkdv launch");
}

int fa2_backward_dq(const float* q, const float* k, const float* v, const float* dout, const float* lse,
                    const float* delta, float* dq, int B, int H, int S, int D, void* stream) {
    int rc;
    if ((rc = check_shape(B, H, S, D)) || (rc = check_ptrs({q, k, v, dout, lse, delta, dq}))) return rc;
    return hip_status(
        fa2::launch_bwd_dq_f16(D, q, k, v, dout, lse, delta, dq, B * H, S, static_cast<hipStream_t>(stream)),
        "fa2_backward_dq launch");
}

int fa2_naive_forward(const float* q, const float* k, const float* v, float* o, float* lse, float* scores, int B,
                      int H, int S, int D, void* stream) {
    int rc;
    if ((rc = check_shape(B, H, S, D)) || (rc = check_ptrs({q, k, v, o, scores}))) return rc;
    return hip_status(fa2::launch_vanilla_forward(D, q, k, v, o, lse, scores, B * H, S, static_cast<hipStream_t>(stream)),
                      "fa2_naive_forward launch");
}

int fa2_fa1_forward(const float* q, const float* k, const float* v, float* o, float* l, float* m, int B, int H, int S,
                    int D, void* stream) {
    int rc;
    if ((rc = check_shape(B, H, S, D)) || (rc = check_ptrs({q, k, v, o, l, m}))) return rc;
    return hip_status(fa2::launch_fa1_forward(D, q, k, v, o, l, m, B * H, S, static_cast<hipStream_t>(stream)),
                      "fa2_fa1_forward launch");
}

int fa2_backward_dq_delta(const float* q, const float* k, const float* v, const float* o, const float* dout,
                          const float* lse, float* delta, float* dq, int B, int H, int S, int D, void* stream) {
    int rc;
    if ((rc = check_shape(B, H, S, D)) || (rc = check_ptrs({q, k, v, o, dout, lse, delta, dq}))) return rc;
    return hip_status(fa2::launch_bwd_dq_delta_f16(D, q, k, v, o, dout, lse, delta, dq, B * H, S,
                                                   static_cast<hipStream_t>(stream)),
                      "fa2_backward_dq_delta launch");
}

}  // extern "C"

// ---------------------------------------------------------------------------
// host-pointer API (+ B*H sharding over devices)
// ---------------------------------------------------------------------------
namespace {

struct HostJob {
    // host tensors (full) and this shard's head range
    const float* in[6] = {};  // q k v o dout lse
    float* out[5] = {};       // o lse | dq dk dv
    int heads0 = 0, nheads = 0, S = 0, D = 0, precision = 0, device = 0, pool = 0;
    bool backward = false;
    float ms = 0.f;
    int rc = FA2_OK;
    std::string err;
};

// Device scratch of the host-pointer API, kept between calls (grow-only) instead of a
// hipMalloc / hipFree per tensor per call: the allocations and frees cost more than
// the kernels at C3.  One pool per (device, shard slot); a call holds its pool's lock
// for its duration.  fa2_host_release() frees them.
struct DevPool {
    std::mutex mu;
    int device = -1;
    void* p = nullptr;
    size_t bytes = 0;
    // streams (compute, H2D, D2H) and events of the pipeline, made once per pool:
    // creating them per call cost ~10 ms of a 15 ms C3 forward call
    int sdev = -1;
    hipStream_t sc = nullptr, si = nullptr, so = nullptr;
    std::vector<hipEvent_t> ev;
    void drop_streams() {
        for (auto e : ev) (void)hipEventDestroy(e);
        ev.clear();
        for (hipStream_t* s : {&sc, &si, &so})
            if (*s) (void)hipStreamDestroy(*s), *s = nullptr;
        sdev = -1;
    }
};
constexpr int kPools = 64;
DevPool g_pools[kPools];

int pool_acquire(DevPool& pl, int device, size_t bytes, char** base) {
    if (pl.p && (pl.bytes < bytes || pl.device != device)) {
        const int prev = pl.device;
        (void)hipSetDevice(prev);
        (void)hipFree(pl.p);
        (void)hipSetDevice(device);
        pl.p = nullptr;
        pl.bytes = 0;
    }
    if (!pl.p) {
        int rc;
        if ((rc = hip_status(hipMalloc(&pl.p, bytes), "hipMalloc"))) return rc;
        pl.bytes = bytes;
        pl.device = device;
    }
    *base = static_cast<char*>(pl.p);
    return FA2_OK;
}

// One shard on one device, as a head-chunked pipeline: H2D of chunk c+1 (this
// thread) overlaps the kernels of chunk c (compute stream) and the D2H of chunk c-1
// (a second host thread: PCIe is full duplex, and a copy from or to pageable memory
// occupies its calling thread).  *ms = the sum of the chunks' kernel times.
int run_shard(HostJob& j) {
    const size_t row = (size_t)j.S * j.D;  // floats per head, [S][D]
    const size_t n = (size_t)j.nheads * row, nl = (size_t)j.nheads * j.S;
    const size_t off = (size_t)j.heads0 * row, offl = (size_t)j.heads0 * j.S;
    if (hipSetDevice(j.device) != hipSuccess) return fail(FA2_E_DEVICE, "hipSetDevice failed");
    // tensors: forward q k v | o lse; backward q k v o dout lse | delta dq dk dv
    const int nin = j.backward ? 6 : 3, nout = j.backward ? 3 : 2;
    const int ntens = j.backward ? 10 : 5;
    auto is_vec = [&](int t) { return j.backward ? (t == 5 || t == 6) : t == 4; };
    size_t bytes = 0;
    size_t toff[10];
    for (int t = 0; t < ntens; ++t) {
        toff[t] = bytes;
        bytes += ((is_vec(t) ? nl : n) * 4 + 255) & ~size_t(255);
    }
    DevPool& pl = g_pools[j.pool % kPools];
    std::lock_guard<std::mutex> lock(pl.mu);
    char* base = nullptr;
    int rc;
    if ((rc = pool_acquire(pl, j.device, bytes, &base))) return rc;
    auto dptr = [&](int t) { return reinterpret_cast<float*>(base + toff[t]); };
    // host side of tensor t: inputs then outputs
    auto hin = [&](int t) { return j.in[t]; };
    auto hout = [&](int t) { return j.backward ? j.out[2 + t] : j.out[t]; };
    // device tensor of output t
    auto dout_t = [&](int t) { return j.backward ? dptr(7 + t) : dptr(3 + t); };
    auto out_vec = [&](int t) { return !j.backward && t == 1; };

    // chunks of heads: about 16 MB of each [S][D] tensor per chunk, at most 4
    int nch = (int)std::min<size_t>(4, std::max<size_t>(1, n * 4 / (size_t(16) << 20)));
    if (const int f = fa2::tune_knob("HOST_CHUNKS", 0)) nch = f;  // A/B override
    nch = std::max(1, std::min(nch, j.nheads));
    if (pl.sdev != j.device) {
        if (pl.sdev >= 0) {
            (void)hipSetDevice(pl.sdev);
            pl.drop_streams();
            (void)hipSetDevice(j.device);
        }
        if ((rc = hip_status(hipStreamCreateWithFlags(&pl.sc, hipStreamNonBlocking), "hipStreamCreate")) ||
            (rc = hip_status(hipStreamCreateWithFlags(&pl.si, hipStreamNonBlocking), "hipStreamCreate")) ||
            (rc = hip_status(hipStreamCreateWithFlags(&pl.so, hipStreamNonBlocking), "hipStreamCreate"))) {
            pl.drop_streams();
            return rc;
        }
        pl.sdev = j.device;
    }
    while ((int)pl.ev.size() < 3 * nch) {  // [c]: inputs in, kernels start, kernels end
        hipEvent_t e = nullptr;
        if ((rc = hip_status(hipEventCreate(&e), "hipEventCreate"))) return rc;
        pl.ev.push_back(e);
    }
    DevPool& r = pl;
    std::vector<int> h0(nch + 1);
    for (int c = 0; c <= nch; ++c) h0[c] = (int)((long)j.nheads * c / nch);

    // D2H thread: waits for each chunk's kernels, copies its outputs back.  It blocks
    // on a condition variable until the chunk's kernels are enqueued (no spinning: with
    // one such thread per shard, spinners would compete with the H2D threads for the
    // host cores).
    std::mutex issue_mu;
    std::condition_variable issue_cv;
    int issued = 0;  // chunks whose kernels are enqueued (guarded by issue_mu)
    bool abort = false;
    auto publish = [&](int n, bool ab) {
        {
            std::lock_guard<std::mutex> g(issue_mu);
            if (n > issued) issued = n;
            abort = abort || ab;
        }
        issue_cv.notify_one();
    };
    int out_rc = FA2_OK;
    std::string out_err;
    std::thread d2h([&] {
        if (hipSetDevice(j.device) != hipSuccess) {
            out_rc = fail(FA2_E_DEVICE, "hipSetDevice failed");
            out_err = g_err;
            return;
        }
        for (int c = 0; c < nch; ++c) {
            {
                std::unique_lock<std::mutex> g(issue_mu);
                issue_cv.wait(g, [&] { return issued > c || abort; });
                if (abort) return;
            }
            int e;
            if ((e = hip_status(hipStreamWaitEvent(r.so, r.ev[3 * c + 2], 0), "hipStreamWaitEvent"))) {
                out_rc = e;
                out_err = g_err;
                return;
            }
            const size_t hc = h0[c + 1] - h0[c];
            for (int t = 0; t < nout; ++t) {
                const size_t per = out_vec(t) ? (size_t)j.S : row;
                const size_t ho = (out_vec(t) ? offl : off) + h0[c] * per;
                if ((e = hip_status(hipMemcpyAsync(hout(t) + ho, dout_t(t) + h0[c] * per, hc * per * 4,
                                                   hipMemcpyDeviceToHost, r.so),
                                    "D2H"))) {
                    out_rc = e;
                    out_err = g_err;
                    return;
                }
            }
        }
        if (int e = hip_status(hipStreamSynchronize(r.so), "D2H")) {
            out_rc = e;
            out_err = g_err;
        }
    });
    // error exits: no copy may still read or write the caller's host buffers, nor
    // the pool's device memory, once the pool lock is released and the call returns
    auto drain = [&] {
        for (hipStream_t s : {r.si, r.sc, r.so}) (void)hipStreamSynchronize(s);
    };
    auto stop = [&](int code) {
        publish(0, true);
        d2h.join();
        drain();
        return code;
    };
    for (int c = 0; c < nch; ++c) {
        const int hc = h0[c + 1] - h0[c];
        for (int t = 0; t < nin; ++t) {
            const bool v = j.backward && t == 5;
            const size_t per = v ? (size_t)j.S : row;
            const size_t ho = (v ? offl : off) + h0[c] * per;
            if ((rc = hip_status(hipMemcpyAsync(dptr(t) + h0[c] * per, hin(t) + ho, hc * per * 4, hipMemcpyHostToDevice,
                                                r.si),
                                 "H2D")))
                return stop(rc);
        }
        if ((rc = hip_status(hipEventRecord(r.ev[3 * c], r.si), "hipEventRecord")) ||
            (rc = hip_status(hipStreamWaitEvent(r.sc, r.ev[3 * c], 0), "hipStreamWaitEvent")) ||
            (rc = hip_status(hipEventRecord(r.ev[3 * c + 1], r.sc), "hipEventRecord")))
            return stop(rc);
        const size_t cr = h0[c] * row, cl = (size_t)h0[c] * j.S;
        if (!j.backward)
            rc = fa2_forward(dptr(0) + cr, dptr(1) + cr, dptr(2) + cr, dptr(3) + cr, dptr(4) + cl, 1, hc, j.S, j.D,
                             j.precision, r.sc);
        else
            rc = fa2_backward(dptr(0) + cr, dptr(1) + cr, dptr(2) + cr, dptr(3) + cr, dptr(4) + cr, dptr(5) + cl,
                              dptr(6) + cl, dptr(7) + cr, dptr(8) + cr, dptr(9) + cr, 1, hc, j.S, j.D, j.precision,
                              r.sc);
        if (rc) return stop(rc);
        if ((rc = hip_status(hipEventRecord(r.ev[3 * c + 2], r.sc), "hipEventRecord"))) return stop(rc);
        publish(c + 1, false);
    }
    d2h.join();
    if (out_rc) {
        drain();
        return fail(out_rc, out_err);
    }
    if ((rc = hip_status(hipStreamSynchronize(r.sc), "kernel"))) return rc;
    float ms = 0.f;
    for (int c = 0; c < nch; ++c) {
        float x = 0.f;
        (void)hipEventElapsedTime(&x, r.ev[3 * c + 1], r.ev[3 * c + 2]);
        ms += x;
    }
    j.ms = ms;
    return FA2_OK;
}

int run_sharded(HostJob proto, int B, int H, int num_devices, float* kernel_ms) {
    const int total = B * H;
    int ndev = num_devices < 1 ? 1 : num_devices;
    // test-only override HOST_SHARDS_ON_DEVICE0 (fa2_tune_set): every shard runs on
    // device 0, each on its own thread and stream, so a one-GPU box exercises the
    // non-zero head offsets of an N-way split
    const bool one_device = fa2::tune_knob("HOST_SHARDS_ON_DEVICE0", 0) != 0;
    const int avail = fa2_device_count();
    if (avail < (one_device ? 1 : ndev)) return fail(FA2_E_INVALID, "num_devices exceeds the visible devices");
    if (ndev > total) ndev = total;
    std::vector<HostJob> jobs(ndev, proto);
    for (int g = 0; g < ndev; ++g) {
        fa2_shard_range(total, ndev, g, &jobs[g].heads0, &jobs[g].nheads);
        jobs[g].device = one_device ? 0 : g;
        jobs[g].pool = g;
    }
    auto body = [](HostJob* j) {
        j->rc = run_shard(*j);
        if (j->rc) j->err = g_err;
    };
    if (ndev == 1) {
        body(&jobs[0]);
    } else {
        std::vector<std::thread> th;
        for (int g = 0; g < ndev; ++g) th.emplace_back(body, &jobs[g]);
        for (auto& t : th) t.join();
    }
    float mx = 0.f;
    for (auto& j : jobs) {
        if (j.rc) return fail(j.rc, "device " + std::to_string(j.device) + ": " + j.err);
        mx = std::max(mx, j.ms);
    }
    if (kernel_ms) *kernel_ms = mx;
    return FA2_OK;
}

}  // namespace

extern "C" {

int fa2_host_release(void) {
    int dev0 = 0;
    const bool have = hipGetDevice(&dev0) == hipSuccess;
    for (auto& pl : g_pools) {
        std::lock_guard<std::mutex> lock(pl.mu);
        if (pl.sdev >= 0) {
            (void)hipSetDevice(pl.sdev);
            pl.drop_streams();
        }
        if (pl.p) {
            (void)hipSetDevice(pl.device);
            (void)hipFree(pl.p);
            pl.p = nullptr;
            pl.bytes = 0;
        }
    }
    if (have) (void)hipSetDevice(dev0);
    fa2::stream_scratch_release();
    return FA2_OK;
}

int fa2_forward_host(const float* q, const float* k, const float* v, float* o, float* lse, int B, int H, int S, int D,
                     int precision, int num_devices, float* kernel_ms) {
    int rc;
    if ((rc = check_shape(B, H, S, D)) || (rc = check_precision(precision)) || (rc = check_ptrs({q, k, v, o, lse})))
        return rc;
    HostJob j;
    j.in[0] = q; j.in[1] = k; j.in[2] = v;
    j.out[0] = o; j.out[1] = lse;
    j.S = S; j.D = D; j.precision = precision;
    return run_sharded(j, B, H, num_devices, kernel_ms);
}

int fa2_backward_host(const float* q, const float* k, const float* v, const float* o, const float* dout,
                      const float* lse, float* dq, float* dk, float* dv, int B, int H, int S, int D, int precision,
                      int num_devices, float* kernel_ms) {
    int rc;
    if ((rc = check_shape(B, H, S, D)) || (rc = check_precision(precision)) ||
        (rc = check_ptrs({q, k, v, o, dout, lse, dq, dk, dv})))
        return rc;
    HostJob j;
    j.in[0] = q; j.in[1] = k; j.in[2] = v; j.in[3] = o; j.in[4] = dout; j.in[5] = lse;
    j.out[2] = dq; j.out[3] = dk; j.out[4] = dv;
    j.S = S; j.D = D; j.precision = precision; j.backward = true;
    return run_sharded(j, B, H, num_devices, kernel_ms);
}

}  // extern "C"
