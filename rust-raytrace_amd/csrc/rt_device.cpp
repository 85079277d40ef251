// C ABI: device contexts, scene upload to HBM, frame/tile rendering.
// See include/raytrace_amd.h for the contract and the reference interfaces
// these replace.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <strings.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "bvh_build.hpp"
#include "device_layout.hpp"
#include "host_scene.hpp"
#include "launch_api.hpp"

using namespace rtamd;

namespace {

// Schedule knobs of a context (rt_ctx_set_tuning).  The defaults are the
// measured-best settings; nothing is read from the environment,
// so a render's schedule depends only on the scene, the options and these.
enum TuneKey : int {
    kTuneChunkPixels, kTuneBvhLeaf, kTuneLgrid, kTuneLgridRes, kTuneSrc, kTuneSrcOcc, kTunePrefixKb2, kTuneLanes,
    kTuneStaggerGen, kTuneRegions, kTuneSplit, kTuneBStreams, kTuneCam, kTuneDeal, kTuneSpreadBelow, kTunePathGroup,
    kTuneCuMask, kTunePrio, kTuneVerbose, kTuneGridOcc, kTuneCompact, kTuneHalf, kTuneWfBudgetMb, kTuneCamGridRes,
    kTuneAQueue, kTuneTailFuse, kTuneTailWidth, kTuneQTree, kTuneCompose, kTuneHostChunks, kTuneHostFirst, kTuneSparseOut,
    kTuneChainOnCaller, kTuneCopyEngine, kTuneDevJoin, kTuneCount
};
struct TuneDef {
    const char* name;
    int64_t dflt, lo, hi;
};
// -1 in src / src_occ / cam / split: chosen per scene.  Round 5 removed the knobs of
// variants measured slower and off by default (DESIGN.md §9 keeps their rows): fuse,
// lists, lists0, fuse_from, prefix4_kb, cam_prefix_kb, tail_from, tail_max, eager_fold,
// fold_split, bmerge, wave_max, tail_fold, tail_shade, fold_wgs, shade_wgs.
constexpr TuneDef kTune[kTuneCount] = {
    {"chunk_pixels", 0, 0, INT32_MAX},          // wavefront chunk cap (0: what the working-set budget holds at the depth)
    {"bvh_leaf", 0, 0, 8},                       // 0: 2 (4 for a quantised tree beyond the LDS budget)
    {"light_grids", 1, 0, 1},                    // light-view grids for point-light shadow queries
    {"light_grid_res", 0, 0, 4096},              // 0: from the median sphere's angular size
    {"src", -1, -1, 26},                         // nearest-hit sphere source (trace_kernel.hip kSrc*)
    {"src_occ", -1, -1, 26},                     // shadow sphere source
    // LDS prefixes stay <= 150 KB: with the queue counters (<= 8.4 KB at 2048 regions) a
    // workgroup's LDS then fits gfx950's 160 KB
    {"prefix_kb", 64, 1, 150},                   // LDS prefix of the binary (or quantised) tree (KB) for trees beyond LDS
    {"lanes", 1, 1, 8},                          // chunk lanes (each its own streams and working set)
    {"stagger_gen", 1, 0, 64},                   // lanes: chunk c+1 starts after this generation of chunk c
    {"regions", 0, 0, 2048},                     // regions per queue (0: 2 x CUs)
    {"split", -1, -1, 1},                        // 0: every wavefront kernel on one in-order stream (-1: per tree)
    {"bstreams", 2, 1, 4},                       // streams for the shadow + shading kernels
    {"cam", -1, -1, 3},                          // generation 0: 3 the camera's view grid (-1: where built), else per ray
    {"deal", 1, 0, 1},                           // chunk dealing: 1 workgroup-major, 0 workgroup-first
    {"spread_below", 0, 0, INT32_MAX},           // queues below this size are dealt workgroup-first
    {"path_group", 0, 0, 64},                    // path kernel: lanes per pixel (0: auto)
    {"cu_mask", 1, 0, 4},                        // b streams CU-masked (own hardware queue): 1 every CU, 2/3/4 only 3/4, 1/2, 1/4 of them
    {"prio", 1, 0, 1},                           // nearest-hit chain on a high-priority stream (round 4: C3 2.969-2.974
                                                 // vs 2.983-2.998 ms, 8-way share 0.713 vs 0.741 ms, C4 equal; same box)
    {"verbose", 0, 0, 1},                        // print the chosen schedule (and a working set that does not fit) to stderr
    {"grid_occ", 1, 0, 1},                       // shadow kernel without a tree walk when every light has a grid
    {"compact_stack", 1, 0, 1},                  // 32-bit nearest-hit stack entries, 32 of them (src 9; src 6 for half-node trees)
    {"half_nodes", 1, 0, 1},                     // trees beyond LDS: binary16 node bounds for the prefix source (src 5)
    {"wf_budget_mb", 0, 0, INT32_MAX},           // wavefront working set of all lanes together (MB; 0: min(80 GB,
                                                 // 85% of the device's free memory)); chunks are sized to it
    {"cam_grid_res", 0, -1, 4096},               // the camera's view grid: cells per face side (0: from the scene's
                                                 // frame size, -1: no grid); takes effect at the next rt_scene_upload
    {"a_queue", 0, 0, 1},                        // 1: the nearest-hit chain's stream CU-masked (a hardware queue of its
                                                 // own, so another context's frame is never queued behind it)
    {"tail_fuse", -1, -1, 32},                   // > 0: the chains running at generation tail_fuse - 1 of a src-9 frame whose
                                                 // lights all have light-view grids finish in one launch (wf_tail); 0 off, -1 auto
    {"tail_width", 0, 0, 64},                    // ... with this many chains per wave (0: auto)
    {"qtree", 0, 0, 1},                          // 1: trees beyond the f32 tree's LDS budget take the quantised 4-wide
                                                 // tree (src 25 whole in LDS, 26 LDS prefix + L2) for the nearest hit;
                                                 // measured slower than binary16 (C4 55.0 vs 50.4 ms, C5 330 vs 307 ms)
    {"compose", 0, 0, 1},                        // 1: the frame is written row by row by wf_compose from the fold's
                                                 // chain-ordered colours (coalesced stores); 0: per pixel by the
                                                 // camera pass and the fold (C3 3.104-3.123 vs 3.235-3.243 ms with
                                                 // 1: the pass itself takes 113 us, the scattered stores it
                                                 // replaces cost the camera pass and the fold less than that)
    {"host_chunks", 1, 1, 64},                   // rt_render into host memory: at least this many chunks, so the D2H
                                                 // copy of one chunk's rows overlaps the next chunk's generations
    {"host_first", 0, 0, 90},                    // with host_chunks 2: the first chunk's share of the rows in percent
                                                 // (0: equal chunks)
    {"sparse_out", 1, 0, 1},                     // rt_render into host memory, one chunk: copy the frame after the camera
                                                 // pass, then only the 16-pixel segments holding chain pixels (§3.11;
                                                 // C3 BGR 4.00 -> 3.46-3.63 ms, RGB + BGR 8.09-8.17 -> 7.67-7.72 ms)
    {"chain_on_caller", 1, 0, 1},                // 1: a one-lane render's nearest-hit chain runs on the caller's stream
                                                 // itself (no fork / join hop between hardware queues at the start and
                                                 // end of the render; the chain then runs at the caller stream's priority;
                                                 // round 6, same box: 8-way C3 share 0.632-0.633 vs 0.650-0.657 ms, 4-way
                                                 // 0.899 vs 0.926 ms, C3 2.767-2.779 vs 2.788-2.790 ms, C4 equal)
    {"copy_engine", -2, -2, 16},                 // rt_render's device -> host copies of the frame: 0 hipMemcpyAsync on the
                                                 // copy stream, e (1..16) the device's SDMA engine e - 1 driven directly
                                                 // (hsa_amd_memory_async_copy_on_engine), -1 its first four engines in turn,
                                                 // -2 (default) -1 for a row-banded tile (a rank's share: band_stride > 1),
                                                 // 0 otherwise (round 6, same box: C3 8-way share into a page-locked frame
                                                 // BGR 1.02 vs 1.35 ms, RGB + BGR 1.43 vs 1.74 ms with -1; C4 share BGR 7.36
                                                 // vs 8.28 ms; the whole C3 frame BGR 3.65 vs 3.80 ms with 0)
    {"dev_join", 1, 0, 1},                       // 1: the b streams join the chain's stream on the device (a one-wave
                                                 // kernel polling a flag the b stream's last kernel is followed by),
                                                 // 0: through events (a barrier packet on the chain's queue)
};

// The table must follow the enum (a key set by name is read through its enum index): checked
// at compile time for every key.
constexpr bool same_name(const char* a, const char* b) { return *a == *b && (*a == 0 || same_name(a + 1, b + 1)); }
static_assert(same_name(kTune[kTuneChunkPixels].name, "chunk_pixels") && same_name(kTune[kTuneBvhLeaf].name, "bvh_leaf") &&
              same_name(kTune[kTuneLgrid].name, "light_grids") && same_name(kTune[kTuneLgridRes].name, "light_grid_res") &&
              same_name(kTune[kTuneSrc].name, "src") && same_name(kTune[kTuneSrcOcc].name, "src_occ") &&
              same_name(kTune[kTunePrefixKb2].name, "prefix_kb") && same_name(kTune[kTuneLanes].name, "lanes") &&
              same_name(kTune[kTuneStaggerGen].name, "stagger_gen") && same_name(kTune[kTuneRegions].name, "regions") &&
              same_name(kTune[kTuneSplit].name, "split") && same_name(kTune[kTuneBStreams].name, "bstreams") &&
              same_name(kTune[kTuneCam].name, "cam") && same_name(kTune[kTuneDeal].name, "deal") &&
              same_name(kTune[kTuneSpreadBelow].name, "spread_below") && same_name(kTune[kTunePathGroup].name, "path_group") &&
              same_name(kTune[kTuneCuMask].name, "cu_mask") && same_name(kTune[kTunePrio].name, "prio") &&
              same_name(kTune[kTuneVerbose].name, "verbose") && same_name(kTune[kTuneGridOcc].name, "grid_occ") &&
              same_name(kTune[kTuneCompact].name, "compact_stack") && same_name(kTune[kTuneHalf].name, "half_nodes") &&
              same_name(kTune[kTuneWfBudgetMb].name, "wf_budget_mb") && same_name(kTune[kTuneCamGridRes].name, "cam_grid_res") &&
              same_name(kTune[kTuneAQueue].name, "a_queue") && same_name(kTune[kTuneTailFuse].name, "tail_fuse") &&
              same_name(kTune[kTuneTailWidth].name, "tail_width") && same_name(kTune[kTuneQTree].name, "qtree") &&
              same_name(kTune[kTuneCompose].name, "compose") && same_name(kTune[kTuneHostChunks].name, "host_chunks") &&
              same_name(kTune[kTuneHostFirst].name, "host_first") && same_name(kTune[kTuneSparseOut].name, "sparse_out") &&
              same_name(kTune[kTuneChainOnCaller].name, "chain_on_caller") &&
              same_name(kTune[kTuneCopyEngine].name, "copy_engine") && same_name(kTune[kTuneDevJoin].name, "dev_join"),
              "kTune[] out of step with TuneKey");

}  // namespace

namespace {

// Host threads that move pinned staging slices into the caller's pageable
// buffer (rt_render): created once per context, so a frame's copy does not pay
// thread start-up per slice.  run() shares any job of parts (the sparse copies'
// row scatter) the same way.  copy() splits one memcpy into kParts parts
// shared by the workers and the calling thread (one thread copies pinned ->
// pageable memory at ~20-28 GB/s, below the DMA's 56 GB/s).  Workers spin
// briefly for the next slice before sleeping, so consecutive slices of a frame
// do not pay a wake-up each.
//
// Each job is published as a snapshot under m_: a worker copies the job's
// fields under the mutex and counts itself in active_ before it takes parts,
// and copy() publishes (and resets the part counters) only once active_ is 0,
// i.e. no worker can still be inside the previous job's part loop.  So a
// worker never mixes two jobs' fields and never claims a part of a job it did
// not snapshot.
class HostCopyPool {
public:
    ~HostCopyPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        for (std::thread& t : th_) t.join();
    }
    void copy(void* to, const void* from, size_t len) {
        const size_t parts = std::max<size_t>(1, std::min<size_t>(kParts, len >> 20));   // >= 1 MiB each
        if (parts == 1) { std::memcpy(to, from, len); return; }
        post(Job{static_cast<uint8_t*>(to), static_cast<const uint8_t*>(from), len, parts, (len + parts - 1) / parts, nullptr});
    }
    // fn(0 .. parts-1), shared by the workers and the calling thread
    void run(size_t parts, const std::function<void(size_t)>& fn) {
        if (parts == 0) return;
        if (parts == 1) { fn(0); return; }
        post(Job{nullptr, nullptr, 0, parts, 0, &fn});
    }
    static constexpr size_t kParts = 8;

private:
    struct Job {
        uint8_t* to = nullptr;
        const uint8_t* from = nullptr;
        size_t len = 0, parts = 0, step = 0;
        const std::function<void(size_t)>* fn = nullptr;   // else a memcpy in parts
    };
    void post(const Job& j) {
        if (th_.empty()) start();
        if (th_.empty()) { next_.store(0, std::memory_order_relaxed); work(j); return; }
        const size_t parts = j.parts;
        {
            std::unique_lock<std::mutex> lk(m_);
            idle_.wait(lk, [&] { return active_ == 0; });    // every worker has left the previous job
            job_ = j;
            next_.store(0, std::memory_order_relaxed);
            done_.store(0, std::memory_order_relaxed);
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        work(j);
        while (done_.load(std::memory_order_acquire) != parts) std::this_thread::yield();
    }

    void start() {
        const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        const unsigned n = std::min<unsigned>(kParts - 1, hw > 1 ? hw - 1 : 1u);
        for (unsigned i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
    }
    void work(const Job& j) {           // take parts of job j until none is left
        for (;;) {
            const size_t q = next_.fetch_add(1, std::memory_order_relaxed);
            if (q >= j.parts) return;
            if (j.fn) {
                (*j.fn)(q);
            } else {
                const size_t a = q * j.step, b = std::min(j.len, a + j.step);
                if (a < b) std::memcpy(j.to + a, j.from + a, b - a);
            }
            done_.fetch_add(1, std::memory_order_release);
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            // spin at most ~200 us for the next slice (the DMA of one slice takes ~150 us), then sleep
            const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(200);
            while (gen_.load(std::memory_order_acquire) == seen && std::chrono::steady_clock::now() < until)
                std::this_thread::yield();
            Job j;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || gen_.load(std::memory_order_acquire) != seen; });
                if (stop_) return;
                seen = gen_.load(std::memory_order_acquire);
                j = job_;
                ++active_;
            }
            work(j);
            {
                std::lock_guard<std::mutex> g(m_);
                --active_;
            }
            idle_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, idle_;
    Job job_;                           // the current job (written and read under m_)
    int active_ = 0;                    // workers inside work() (under m_)
    bool stop_ = false;                 // (under m_)
    std::atomic<size_t> next_{0}, done_{0};
    std::atomic<uint64_t> gen_{0};
};

constexpr int kMaxBands = 16;           // row bands of one rt_render copied as they finish
constexpr int kRing = 4;                // pinned staging slices in flight
constexpr size_t kSlice = 8u << 20;     // bytes per staging slice

}  // namespace

struct rt_ctx {
    int device = 0;
    int n_cu = 256;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr;             // start of the last render (its end: render_done, also a timing event)
    void* d_blob = nullptr;
    size_t blob_bytes = 0;
    DevScene dsc{};
    bool has_scene = false;
    bool deep_bvh4 = false;          // the 4-wide tree could overflow the traversal stack: binary tree only
    bool short_stack = false;        // binary tree fits the compact nearest-hit stack (16-bit codes, depth <= 32)
    bool short_stack18 = false;      // ... with 18-bit codes (the binary16 prefix source, src 6)
    bool q4_ok = false;              // the quantised 4-wide tree was built (DevScene::q4)
    bool all_lights_gridded = false; // every light is a point light with a light-view grid
    unsigned long long* d_counters = nullptr;
    double* d_srgb = nullptr;         // the 255 sRGB thresholds (path kernel)
    void* d_path = nullptr;           // path kernel recursion stack (PathStack)
    size_t path_bytes = 0;
    float* d_rgb = nullptr;
    size_t rgb_cap = 0;
    uint8_t* d_bgr = nullptr;
    size_t bgr_cap = 0;
    uint64_t last_pixels = 0;
    bool last_timed = false;
    bool ev0_set = true;                   // ev0 was recorded at the start of the last render
    // rt_render_device without RT_TIME_KERNELS / RT_COUNT_WORK: no ev0 (rt_stats.kernel_ms 0): the
    // marker between consecutive renders on the caller's stream cost ~4-6 us of device time per
    // frame (8-way C3 share 0.655-0.656 vs 0.659-0.662 ms, C3 2.800 vs 2.812 ms, same box)
    bool skip_ev0 = false;
    hipStream_t last_stream = nullptr;
    // Wavefront lanes: each owns a stream and a working set (grown on demand,
    // kept across renders).  Row chunks of a render are dealt round-robin over
    // the lanes; chunk c+1 starts once chunk c has passed its bulk generations,
    // so its big launches overlap chunk c's latency-bound tail.
    struct Lane {
        hipStream_t s = nullptr;
        std::vector<hipStream_t> sb;       // shadow + shading kernels of the generations
        hipEvent_t mark = nullptr, done = nullptr;
        std::vector<hipEvent_t> b_done;    // one per sb stream
        std::vector<hipEvent_t> near_done; // per generation: nearest-hit kernel finished (s -> sb)
        void* mem = nullptr;
        size_t bytes = 0;
        WfBufs b{};
        uint64_t* dj = nullptr;            // device-side join flags (kDjWords words, zeroed once)
        uint64_t dj_n = 0;                 // the last join number handed out on them
        uint64_t* dj_err = nullptr;        // page-locked: a join gave up (host address; dj_err_dev the device's)
        uint64_t* dj_err_dev = nullptr;
    };
    std::vector<Lane> lanes;
    // RT_TIME_KERNELS: launch intervals accumulated since the last harvest
    std::vector<hipEvent_t> tev;
    int t_used = 0;
    std::vector<LaunchInterval> tint;
    hipEvent_t fork = nullptr;
    bool wf_used = false;
    // a one-chunk wavefront render leaves its tally (ray counts, per-generation queue sizes) to
    // the first rt_ctx_stats / rt_ctx_generation_counts after it (flush_tally): not on the chain
    struct PendingTally {
        bool on = false;
        bool zero = false;                 // the render left the counters to be cleared before the tally
        FrameParams fp{};
        WfBufs b{};
        int n_lights = 0, gens = 0;
    } tally;
    uint32_t scene_spp = 1;           // the uploaded scene's Options.antialias (rt_render_opts.spp = 0)
    hipEvent_t render_done = nullptr; // end of the last render on its stream: the next one waits for it
    bool render_pending = false;
    hipStream_t done_stream = nullptr;     // the stream render_done was recorded on
    uint32_t last_spp_traced = 1;     // chain schedules trace one of spp identical centre-jitter samples
    uint32_t last_chunks = 0;         // wavefront chunks of the last render (0: other schedules)
    // rt_render: pinned staging slices for the device -> host copy of the outputs, a copy
    // stream that waits for each finished row band, and the host threads that empty the slices
    void* pin[kRing] = {};
    size_t pin_cap = kSlice;               // bytes per staging slice (larger for rows wider than kSlice)
    hipEvent_t pin_ev[kRing] = {};
    hipStream_t copy_stream = nullptr;
    bool want_bands = false;               // set by rt_render around its render: fold in bands, events after each
    int n_bands = 0;                       // bands of the last render (0: copy after render_done)
    hipEvent_t band_ev[kMaxBands] = {};
    uint32_t band_row0[kMaxBands] = {}, band_nrows[kMaxBands] = {};
    HostCopyPool pool;
    // sparse host copies (tuning sparse_out): device segment bits / row counts /
    // row offsets / packed BGR / packed RGB, the pinned host copies of the first three and of the
    // packed segments, and an event per piece of the packed copy
    bool want_sparse = false;              // set by rt_render around its render
    bool sparse_on = false;                // the last render marked its chain pixels and packed them
    void* d_sp = nullptr;
    size_t sp_cap = 0;
    uint32_t* d_sp_bits = nullptr, *d_sp_cnt = nullptr, *d_sp_off = nullptr;
    uint8_t* d_sp_bgr = nullptr;
    float* d_sp_rgb = nullptr;
    void* h_sp_meta = nullptr;
    size_t h_sp_meta_cap = 0;
    void* h_sp_pk = nullptr;
    size_t h_sp_pk_cap = 0;
    hipEvent_t sp_cam = nullptr, sp_ready = nullptr, cp_done = nullptr;
    static constexpr int kSpRanges = 16;   // row ranges of the packed copy, each scattered as it lands
    hipEvent_t sp_ev[kSpRanges] = {};
    // copies on an SDMA engine (tuning copy_engine): the device's and a CPU agent, the engine, and
    // one completion signal per staging slice / packed range / direct copy batch
    int sdma_state = 0;                    // 0 not set up, 1 usable, -1 unavailable
    bool copy_banded = false;              // the rt_render under way writes a row-banded tile (copy_engine -2)
    bool dj_used = false;                  // a render joined its streams on the device (check_join_error)
    hsa_agent_t hsa_gpu{}, hsa_cpu{};
    uint32_t sdma_avail = 0, sdma_pref = 0, sdma_turn = 0;
    static constexpr int kSdmaSignals = kRing + kSpRanges + 1;
    hsa_signal_t sdma_sig[kSdmaSignals] = {};
    int64_t tune[kTuneCount];
    std::string err;
    rt_ctx() {
        for (int i = 0; i < kTuneCount; ++i) tune[i] = kTune[i].dflt;
        // a device-side join spins while the b streams finish: it needs their kernels to run beside
        // it, which kernel serialisation (rocprofv3 --pmc, AMD_SERIALIZE_KERNEL) does not allow (the
        // join would wait out its 2 s limit): joins through events there
        auto on = [](const char* v) { return v && *v && std::strcmp(v, "0") != 0 && strcasecmp(v, "false") != 0; };
        if (on(std::getenv("ROCPROF_COUNTER_COLLECTION")) || on(std::getenv("AMD_SERIALIZE_KERNEL"))) tune[kTuneDevJoin] = 0;
    }
    int64_t t(TuneKey k) const { return tune[k]; }
};

namespace {

int fail(rt_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    set_thread_error(msg);
    return code;
}

int hip_fail(rt_ctx* c, hipError_t e, const char* what) {
    return fail(c, RT_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(c, expr)                                            \
    do {                                                            \
        hipError_t _e = (expr);                                     \
        if (_e != hipSuccess) return hip_fail((c), _e, #expr);      \
    } while (0)

// No C++ exception crosses the ABI: allocation failures become RT_E_NOMEM.
template <class F>
int guarded(rt_ctx* c, F&& body) {
    try {
        return body();
    } catch (const std::bad_alloc&) {
        return fail(c, RT_E_NOMEM, "host allocation failed");
    } catch (const std::exception& e) {
        return fail(c, RT_E_INVALID, e.what());
    } catch (...) {
        return fail(c, RT_E_INVALID, "unexpected exception");
    }
}

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// counters: [0, 256) rays per shard (megakernel), [256, 512) shadow rays per
// shard, [512, 520) wavefront totals (see WfBufs::totals), [520, 520 + kCntWords)
// per-generation queue sizes summed over chunks
constexpr int kTotals = 2 * kCounterShards;
constexpr int kGenTotals = kTotals + 8;
constexpr int kCounterWords = kGenTotals + kCntWords;
static_assert(kMatPhong == RT_MAT_PHONG && kMatFresnel == RT_MAT_FRESNEL && kMatIndirect == RT_MAT_INDIRECT_PHONG &&
                  kMatTransparent == RT_MAT_TRANSPARENT,
              "DevMaterial::kind mirrors rt_material_kind");
static_assert(kLightArea == RT_LIGHT_AREA, "DevLight::kind mirrors rt_light_kind");
// LDS per traversal workgroup for staged scene data (1024 threads, two resident per CU)
constexpr size_t kLdsBudget = 72 * 1024;
constexpr uint64_t kWfBudget = 80ull << 30;     // default wavefront working set per lane (of 288 GB HBM)
// device memory a working set must leave free: the runtime's per-queue scratch
// (up to 32 waves x 256 CUs x 64 lanes x ~600 B per queue, for several queues)
constexpr size_t kRuntimeHeadroom = 4ull << 30;

// The b streams need hardware queues of their own: HIP deals streams over a
// few shared queues (GPU_MAX_HW_QUEUES), and two streams on one queue run
// strictly in submission order.  A CU-masked stream (mask = every CU) gets a
// dedicated queue.  Created on demand: every extra hardware queue costs the
// firmware scheduler, measurably slowing the others.
int ensure_bstreams(rt_ctx* c, rt_ctx::Lane& M, int nb) {
    std::vector<uint32_t> mask((c->n_cu + 31) / 32, 0u);
    const int keep = 5 - static_cast<int>(std::max<int64_t>(1, c->t(kTuneCuMask)));   // of every 4 CUs
    for (int cu = 0; cu < c->n_cu; ++cu)
        if (cu % 4 < keep) mask[cu / 32] |= 1u << (cu % 32);
    while (static_cast<int>(M.sb.size()) < nb) {
        hipStream_t s = nullptr;
        if (c->t(kTuneCuMask) == 0 ||
            hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(mask.size()), mask.data()) != hipSuccess) {
            (void)hipGetLastError();
            HIP_TRY(c, hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        }
        M.sb.push_back(s);
        hipEvent_t e = nullptr;
        HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        M.b_done.push_back(e);
    }
    return RT_OK;
}

// Free every lane (streams, events, working set) once its work is done.  Used
// by rt_ctx_destroy, by rt_ctx_set_tuning when a key that shapes the streams
// (cu_mask, prio) changes, and before a render retries with smaller chunks.
void drop_lane_memory(rt_ctx::Lane& L) {
    if (L.s) (void)hipStreamSynchronize(L.s);
    for (hipStream_t x : L.sb) if (x) (void)hipStreamSynchronize(x);
    if (L.mem) (void)hipFree(L.mem);
    L.mem = nullptr;
    L.bytes = 0;
}

void drop_lanes(rt_ctx* c) {
    for (auto& L : c->lanes) {
        drop_lane_memory(L);
        if (L.mark) (void)hipEventDestroy(L.mark);
        if (L.done) (void)hipEventDestroy(L.done);
        for (hipEvent_t e : L.b_done) if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : L.near_done) if (e) (void)hipEventDestroy(e);
        if (L.s) (void)hipStreamDestroy(L.s);
        for (hipStream_t x : L.sb) if (x) (void)hipStreamDestroy(x);
        if (L.dj) (void)hipFree(L.dj);
        if (L.dj_err) (void)hipHostFree(L.dj_err);
    }
    c->lanes.clear();
}

// Working-set bytes per pixel slot of a chunk (ensure_wf's sections, per slot):
// two queues, one shade-record array and one level array per lit generation,
// terminals and level counts, the chain's pixel, the pixel map and the chain colours.
uint64_t wf_bytes_per_slot(uint64_t levels) {
    return 2ull * 8 * 8 + levels * (7 * 8 + 4 * 4) + levels * (4 * 8 + 4) + (3 * 8 + 1) + 4 + 4 + 16;
}

// Default working-set budget of a render (all lanes): 85% of what the device
// has free plus what this context's lanes already hold, at most kWfBudget.
uint64_t default_wf_budget(rt_ctx* c) {
    size_t fr = 0, total = 0;
    uint64_t held = 0;
    for (const auto& L : c->lanes) held += L.bytes;
    if (hipMemGetInfo(&fr, &total) != hipSuccess) {
        (void)hipGetLastError();
        return kWfBudget;
    }
    return std::min<uint64_t>(kWfBudget, static_cast<uint64_t>(0.85 * static_cast<double>(fr + held)));
}

int ensure_lanes(rt_ctx* c, int n) {
    while (static_cast<int>(c->lanes.size()) < n) {
        rt_ctx::Lane L;
        c->lanes.push_back(L);
        rt_ctx::Lane& M = c->lanes.back();
        // prio: the nearest-hit chain (the critical path) on a high-priority stream
        int lo = 0, hi = 0;
        std::vector<uint32_t> all((c->n_cu + 31) / 32, 0u);
        for (int cu = 0; cu < c->n_cu; ++cu) all[cu / 32] |= 1u << (cu % 32);
        if (c->t(kTunePrio) && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess) {
            HIP_TRY(c, hipStreamCreateWithPriority(&M.s, hipStreamNonBlocking, hi));
        } else if (c->t(kTuneAQueue) == 0 ||
                   hipExtStreamCreateWithCUMask(&M.s, static_cast<uint32_t>(all.size()), all.data()) != hipSuccess) {
            (void)hipGetLastError();
            HIP_TRY(c, hipStreamCreateWithFlags(&M.s, hipStreamNonBlocking));
        }
        HIP_TRY(c, hipEventCreateWithFlags(&M.mark, hipEventDisableTiming));
        HIP_TRY(c, hipEventCreateWithFlags(&M.done, hipEventDisableTiming));
        M.near_done.assign(kMaxGenerations, nullptr);
        for (hipEvent_t& e : M.near_done) HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIP_TRY(c, hipMalloc(reinterpret_cast<void**>(&M.dj), kDjWords * sizeof(uint64_t)));
        HIP_TRY(c, hipMemset(M.dj, 0, kDjWords * sizeof(uint64_t)));
        HIP_TRY(c, hipHostMalloc(reinterpret_cast<void**>(&M.dj_err), sizeof(uint64_t), hipHostMallocMapped));
        *M.dj_err = 0;
        HIP_TRY(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&M.dj_err_dev), M.dj_err, 0));
    }
    return RT_OK;
}

// Carve a lane's wavefront working set for chunks of up to `cap` pixels: every
// queue and shade-record array is G regions of R entries; the shade records
// have one such array per lit generation (`levels` = max_depth + 1).
int ensure_wf(rt_ctx* c, rt_ctx::Lane& L, uint32_t cap, uint32_t G, uint32_t R, uint32_t levels) {
    WfBufs& b = L.b;
    const uint64_t q = static_cast<uint64_t>(G) * R;   // queue capacity (>= generation-0 slots)
    const uint64_t capa = align_up(q, 64);               // per-chain arrays (chain = generation-0 record entry)
    // section sizes (device_layout.hpp, WfBufs)
    const uint64_t s_queue = 2ull * 8 * q * 8;
    const uint64_t s_rec = static_cast<uint64_t>(levels) * q * (7 * 8 + 4 * 4);
    const uint64_t s_lev = static_cast<uint64_t>(levels) * capa * (4 * 8 + 4);
    const uint64_t s_term = capa * (3 * 8 + 1);
    const uint64_t s_reg = static_cast<uint64_t>(kMaxGenerations) * G * 4;
    const uint64_t s_cpix = q * 4;
    const uint64_t s_pmap = static_cast<uint64_t>(cap) * 4;
    const uint64_t s_ccol = capa * 16;
    uint64_t off = align_up(s_queue, 256);
    b.o_rec = off; off = align_up(off + s_rec, 256);
    b.o_lev = off; off = align_up(off + s_lev, 256);
    b.o_term = off; off = align_up(off + s_term, 256);
    b.o_rq = off; off = align_up(off + s_reg, 256);
    b.o_rs = off; off = align_up(off + s_reg, 256);
    b.o_cpix = off; off = align_up(off + s_cpix, 256);
    b.o_pmap = off; off = align_up(off + s_pmap, 256);
    b.o_ccol = off; off = align_up(off + s_ccol, 256);
    if (off > L.bytes) {
        if (L.mem) {
            // every render still using it is done (its chain may have run on a caller's stream)
            if (c->render_pending) (void)hipEventSynchronize(c->render_done);
            (void)hipStreamSynchronize(L.s);
            for (hipStream_t x : L.sb) (void)hipStreamSynchronize(x);
            (void)hipFree(L.mem);
        }
        L.mem = nullptr;
        L.bytes = 0;
        // ask only for what the device has free, less the runtime's scratch headroom: a request
        // beyond it is answered without hipMalloc (the runtime has crashed inside a failing
        // hipMalloc of a few hundred GB, seen with an explicit oversized wf_budget_mb), and a
        // working set that took the last free bytes would leave nothing for the scratch the
        // runtime allocates per hardware queue at a kernel's first launch there.  The free
        // memory is the device's: other contexts and processes count, so the caller's halving
        // of the chunks is reported under tuning verbose and in rt_stats.chunks.
        size_t fr = 0, total = 0;
        if (hipMemGetInfo(&fr, &total) == hipSuccess && (off > fr || fr - off < kRuntimeHeadroom)) {
            if (c->t(kTuneVerbose))
                std::fprintf(stderr, "rtamd: working set of %llu MB does not fit %llu MB free (less %llu MB headroom): "
                             "halving the chunk\n", static_cast<unsigned long long>(off >> 20),
                             static_cast<unsigned long long>(fr >> 20), static_cast<unsigned long long>(kRuntimeHeadroom >> 20));
            return fail(c, RT_E_NOMEM, "wavefront working set of " + std::to_string(off >> 20) + " MB does not fit (" +
                                           std::to_string(fr >> 20) + " MB free)");
        }
        (void)hipGetLastError();
        const hipError_t e = hipMalloc(&L.mem, off);
        if (e == hipErrorOutOfMemory) {          // the caller retries with smaller chunks
            (void)hipGetLastError();
            L.mem = nullptr;
            if (c->t(kTuneVerbose))
                std::fprintf(stderr, "rtamd: hipMalloc of %llu MB failed: halving the chunk\n",
                             static_cast<unsigned long long>(off >> 20));
            return fail(c, RT_E_NOMEM, "wavefront working set of " + std::to_string(off >> 20) + " MB does not fit");
        }
        if (e != hipSuccess) return hip_fail(c, e, "hipMalloc(wavefront working set)");
        L.bytes = off;
    }
    b.mem = static_cast<unsigned char*>(L.mem);
    b.totals = c->d_counters + kTotals;
    b.gen_totals = c->d_counters + kGenTotals;
    b.qcap = q;
    b.cap = cap;
    b.capa = static_cast<uint32_t>(capa);
    b.levels = levels;
    b.G = G;
    b.R = R;
    return RT_OK;
}

double significance(const rt_color& c) { return c.r + c.g + c.b; }   // color.rs:637-639

}  // namespace

extern "C" {

int rt_device_count(int* n) {
    if (!n) return RT_E_INVALID;
    *n = 0;
    int k = 0;
    hipError_t e = hipGetDeviceCount(&k);
    if (e != hipSuccess) { *n = 0; return RT_OK; }
    *n = k;
    return RT_OK;
}

static int warm_streams(rt_ctx* c, const std::vector<hipStream_t>& ss);

int rt_ctx_create(int device, rt_ctx** out) {
    if (!out) return RT_E_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
        return fail(nullptr, RT_E_NODEVICE, "no HIP device " + std::to_string(device));
    auto* c = new (std::nothrow) rt_ctx();
    if (!c) return RT_E_NOMEM;
    c->device = device;
    if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || c->n_cu < 1)
        c->n_cu = 256;
    auto cleanup = [&](int rc) { rt_ctx_destroy(c); return rc; };
    if (hipSetDevice(device) != hipSuccess) return cleanup(fail(nullptr, RT_E_HIP, "hipSetDevice failed"));
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess ||
        hipEventCreateWithFlags(&c->fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreate(&c->render_done) != hipSuccess ||
        hipMalloc(&c->d_counters, kCounterWords * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&c->d_srgb, 255 * sizeof(double)) != hipSuccess ||
        hipMemcpy(c->d_srgb, srgb_average_table(), 255 * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
        upload_srgb_table(srgb_average_table()) != hipSuccess)
        return cleanup(fail(nullptr, RT_E_HIP, "context initialisation failed"));
    // the kernels' code objects load at their first launch: here, not in the first render
    if (warm_streams(c, {c->stream}) != RT_OK) return cleanup(fail(nullptr, RT_E_HIP, "context warm-up failed"));
    *out = c;
    return RT_OK;
}

void rt_ctx_destroy(rt_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->render_pending) (void)hipEventSynchronize(c->render_done);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->d_blob) (void)hipFree(c->d_blob);
    if (c->d_counters) (void)hipFree(c->d_counters);
    if (c->d_srgb) (void)hipFree(c->d_srgb);
    if (c->d_path) (void)hipFree(c->d_path);
    if (c->d_rgb) (void)hipFree(c->d_rgb);
    if (c->d_bgr) (void)hipFree(c->d_bgr);
    drop_lanes(c);
    for (hipEvent_t e : c->tev) (void)hipEventDestroy(e);
    if (c->render_done) (void)hipEventDestroy(c->render_done);
    if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
    for (int i = 0; i < kRing; ++i) {
        if (c->pin[i]) (void)hipHostFree(c->pin[i]);
        if (c->pin_ev[i]) (void)hipEventDestroy(c->pin_ev[i]);
    }
    for (hipEvent_t e : c->band_ev) if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->sp_ev) if (e) (void)hipEventDestroy(e);
    if (c->sp_cam) (void)hipEventDestroy(c->sp_cam);
    if (c->sp_ready) (void)hipEventDestroy(c->sp_ready);
    if (c->cp_done) (void)hipEventDestroy(c->cp_done);
    if (c->d_sp) (void)hipFree(c->d_sp);
    if (c->sdma_state == 1) {
        for (hsa_signal_t sg : c->sdma_sig)
            if (sg.handle) (void)hsa_signal_destroy(sg);
        (void)hsa_shut_down();             // balances sdma_setup's hsa_init
    }
    if (c->h_sp_meta) (void)hipHostFree(c->h_sp_meta);
    if (c->h_sp_pk) (void)hipHostFree(c->h_sp_pk);
    if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
    if (c->fork) (void)hipEventDestroy(c->fork);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* rt_last_error(const rt_ctx* c) { return c ? c->err.c_str() : thread_error(); }

int rt_light_grid_candidates(const rt_scene* s, int light, int resolution, const double* points, uint32_t n_points,
                             int32_t* counts, int32_t* ids, size_t cap, int64_t* info) {
    if (!s || (n_points && (!points || !counts)) || (cap && !ids)) return RT_E_INVALID;
    if (light < 0 || light >= static_cast<int>(s->lights.size()) || resolution < 0 || resolution > 4096)
        return RT_E_INVALID;
    try {
        std::vector<DevSphere> spheres;
        std::vector<double> srad;
        std::vector<int32_t> obj;
        double extent = 0.0;
        for (size_t i = 0; i < s->objects.size(); ++i) {
            const rt_object& o = s->objects[i];
            if (o.shape != RT_SHAPE_SPHERE) continue;
            spheres.push_back(DevSphere{o.geom[0], o.geom[1], o.geom[2], o.geom[3] * o.geom[3]});
            srad.push_back(o.geom[3]);
            obj.push_back(static_cast<int32_t>(i));
            const double r = std::fabs(o.geom[3]);
            for (int k = 0; k < 3; ++k)
                for (double v : {o.geom[k] - r, o.geom[k] + r})
                    if (std::isfinite(v)) extent = std::max(extent, std::fabs(v));
        }
        std::vector<DevLight> lights;
        for (const rt_light& l : s->lights) {
            DevLight d{};
            for (int k = 0; k < 9; ++k) d.v[k] = l.v[k];
            d.kind = l.kind;
            lights.push_back(d);
        }
        const LightGridResult lg = build_light_grids(spheres, srad, lights, 1e-5 * (1.0 + extent), resolution);
        if (info) {
            info[0] = lg.grids[light].R;
            int64_t cells = 0;
            for (int f = 0; f < 6; ++f) cells += static_cast<int64_t>(lg.grids[light].fw[f]) * lg.grids[light].fh[f];
            info[1] = cells;
            info[2] = static_cast<int64_t>(lg.ent.size());
        }
        std::vector<int32_t> cand;
        size_t used = 0;
        for (uint32_t i = 0; i < n_points; ++i) {
            if (!light_grid_candidates(lg, light, points + 3 * i, cand)) { counts[i] = -1; continue; }
            counts[i] = static_cast<int32_t>(cand.size());
            for (int32_t k : cand) {
                if (used == cap) return fail(nullptr, RT_E_INVALID, "candidate buffer too small");
                ids[used++] = obj[k];
            }
        }
        return RT_OK;
    } catch (const std::exception& e) {
        return fail(nullptr, RT_E_NOMEM, e.what());
    }
}

// The view grid's automatic resolution: a cell about 8 x 8 pixels of the scene's frame.
static int view_grid_res(const rt_scene* s, int64_t forced) {
    if (forced > 0) return static_cast<int>(forced);
    const double* M = s->camera.matrix;
    const double imd = std::sqrt(M[2] * M[2] + M[5] * M[5] + M[8] * M[8]);
    const double side = static_cast<double>(std::max(std::max(s->width, s->height), 64u));
    return std::isfinite(imd) ? static_cast<int>(std::lround(std::clamp(imd * side / 8.0, 16.0, 2048.0))) : 64;
}
constexpr size_t kViewGridEntries = size_t{32} << 20;
// the view grid's list entries: at most 32 M, and about 4096 per sphere (C3 holds 395 per sphere)
static size_t view_grid_cap(size_t n_spheres) { return std::min(kViewGridEntries, (size_t{1} << 20) + 4096 * n_spheres); }

int rt_view_grid_candidates(const rt_scene* s, int resolution, const double* dirs, uint32_t n_dirs, int32_t* counts,
                            int32_t* ids, float* nears, size_t cap, int64_t* info) {
    if (!s || (n_dirs && (!dirs || !counts)) || (cap && (!ids || !nears)) || resolution < 0 || resolution > 4096)
        return RT_E_INVALID;
    try {
        std::vector<DevSphere> spheres;
        std::vector<double> srad;
        std::vector<int32_t> obj;
        double extent = 0.0;
        for (size_t i = 0; i < s->objects.size(); ++i) {
            const rt_object& o = s->objects[i];
            if (o.shape != RT_SHAPE_SPHERE) continue;
            spheres.push_back(DevSphere{o.geom[0], o.geom[1], o.geom[2], o.geom[3] * o.geom[3]});
            srad.push_back(o.geom[3]);
            obj.push_back(static_cast<int32_t>(i));
            const double r = std::fabs(o.geom[3]);
            for (int k = 0; k < 3; ++k)
                for (double v : {o.geom[k] - r, o.geom[k] + r})
                    if (std::isfinite(v)) extent = std::max(extent, std::fabs(v));
        }
        const LightGridResult g = build_view_grid(spheres, srad, s->camera.position, 1e-5 * (1.0 + extent),
                                                  view_grid_res(s, resolution), view_grid_cap(spheres.size()));
        const DevLightGrid& G = g.grids[0];
        if (info) {
            info[0] = G.R;
            int64_t cells = 0;
            for (int f = 0; f < 6; ++f) cells += static_cast<int64_t>(G.fw[f]) * G.fh[f];
            info[1] = cells;
            info[2] = static_cast<int64_t>(g.ent.size());
        }
        size_t used = 0;
        auto put = [&](const DevLgEntry& e) {
            if (used == cap) throw std::length_error("candidate buffer too small");
            ids[used] = obj[e.sph];
            nears[used++] = e.near;
        };
        for (uint32_t i = 0; i < n_dirs; ++i) {
            const size_t before = used;
            for (uint32_t e = G.always_begin; e < G.always_end; ++e) put(g.ent[e]);
            // the device's lookup (nearest_cgrid): f32 direction, dominant axis, clamped cell
            const float dx = static_cast<float>(dirs[3 * i]), dy = static_cast<float>(dirs[3 * i + 1]),
                        dz = static_cast<float>(dirs[3 * i + 2]);
            const float ax = std::fabs(dx), ay = std::fabs(dy), az = std::fabs(dz);
            const int fa = (ax >= ay && ax >= az) ? 0 : (ay >= az ? 1 : 2);
            const float da = fa == 0 ? dx : fa == 1 ? dy : dz;
            const float db = fa == 0 ? dy : fa == 1 ? dz : dx;
            const float dc = fa == 0 ? dz : fa == 1 ? dx : dy;
            if (G.R <= 0 || !(std::fabs(da) > 0.0f && std::fabs(da) < 3.0e38f)) { counts[i] = -1; used = before; continue; }
            const int f = 2 * fa + (da < 0.0f ? 1 : 0);
            const float inv = 1.0f / std::fabs(da);
            const float R = static_cast<float>(G.R);
            const int ci = std::min(std::max(static_cast<int>(std::floor((db * inv + 1.0f) * 0.5f * R)), 0), G.R - 1);
            const int cj = std::min(std::max(static_cast<int>(std::floor((dc * inv + 1.0f) * 0.5f * R)), 0), G.R - 1);
            const int li = ci - G.fx0[f], lj = cj - G.fy0[f];
            if (li >= 0 && lj >= 0 && li < G.fw[f] && lj < G.fh[f]) {
                const uint32_t cell = G.off_base[f] + static_cast<uint32_t>(lj * G.fw[f] + li);
                for (uint32_t e = g.off[cell]; e < g.off[cell + 1]; ++e) put(g.ent[e]);
            }
            counts[i] = static_cast<int32_t>(used - before);
        }
        return RT_OK;
    } catch (const std::length_error& e) {
        return fail(nullptr, RT_E_INVALID, e.what());
    } catch (const std::exception& e) {
        return fail(nullptr, RT_E_NOMEM, e.what());
    }
}

int rt_qtree_nodes(const rt_scene* s, int leaf_max, void* nodes, float* boxes, int32_t* sphere_first,
                   int32_t* sphere_count, size_t cap_nodes, int64_t* info) {
    if (!s || leaf_max < 0 || leaf_max > 8 || (cap_nodes && (!nodes || !boxes || !sphere_first || !sphere_count)))
        return RT_E_INVALID;
    try {
        std::vector<double> sx, sy, sz, srad;
        double extent = 0.0;
        for (const rt_object& o : s->objects) {
            if (o.shape != RT_SHAPE_SPHERE) continue;
            sx.push_back(o.geom[0]); sy.push_back(o.geom[1]); sz.push_back(o.geom[2]); srad.push_back(o.geom[3]);
            const double r = std::fabs(o.geom[3]);
            for (int k = 0; k < 3; ++k)
                for (double v : {o.geom[k] - r, o.geom[k] + r})
                    if (std::isfinite(v)) extent = std::max(extent, std::fabs(v));
        }
        const double pad = 1e-5 * (1.0 + extent);
        // the quantised tree's leaf rule (scene_upload with tuning qtree): 2, or 4 when that tree
        // and the spheres would not fit the LDS budget
        int leaf = leaf_max > 0 ? leaf_max : 2;
        BvhResult bvh = build_sphere_bvh(sx, sy, sz, srad, pad, leaf);
        if (leaf_max == 0 && bvh.nodes.size() * sizeof(DevBvhNode) + sx.size() * (sizeof(DevSphere) + 4) > kLdsBudget)
            bvh = build_sphere_bvh(sx, sy, sz, srad, pad, leaf = 4);
        const Bvh4Result b4 = collapse_bvh4(bvh);
        const int need = bvh4_stack_need(b4);
        const std::vector<DevQNode4> q = need <= kQ4Stack ? quantize_bvh4(b4) : std::vector<DevQNode4>{};
        if (info) { info[0] = static_cast<int64_t>(q.size()); info[1] = need; info[2] = leaf; }
        if (cap_nodes == 0) return RT_OK;                  // a size query: info[] alone
        if (q.size() > cap_nodes) return fail(nullptr, RT_E_INVALID, "node buffer too small");
        if (q.empty()) return RT_OK;
        const int32_t N = b4.n_nodes;
        std::memcpy(nodes, q.data(), q.size() * sizeof(DevQNode4));
        for (size_t i = 0; i < q.size(); ++i)
            for (int k = 0; k < 4; ++k) {
                const int32_t ch = b4.planes[static_cast<size_t>(6) * N + i].i[k];
                for (int a = 0; a < 3; ++a) {
                    boxes[(i * 4 + k) * 6 + a] = ch == kBvh4Empty ? NAN : b4.planes[static_cast<size_t>(2 * a) * N + i].f[k];
                    boxes[(i * 4 + k) * 6 + 3 + a] = ch == kBvh4Empty ? NAN : b4.planes[static_cast<size_t>(2 * a + 1) * N + i].f[k];
                }
                const bool leafc = ch != kBvh4Empty && ch < 0;
                sphere_first[i * 4 + k] = leafc ? (~ch) >> 3 : -1;
                sphere_count[i * 4 + k] = leafc ? ((~ch) & 7) + 1 : 0;
            }
        return RT_OK;
    } catch (const std::exception& e) {
        return fail(nullptr, RT_E_NOMEM, e.what());
    }
}

static int scene_upload(rt_ctx* c, const rt_scene* s) {
    HIP_TRY(c, hipSetDevice(c->device));
    // Every class of the reference except SkyboxBackground (textures) has a
    // device implementation: Phong / Fresnel chains on the wavefront path,
    // the stochastic and branching classes on the path kernel (needs_path).
    if (s->background_kind != RT_BG_SOLID && s->background_kind != RT_BG_SKYBOX)
        return fail(c, RT_E_INVALID, "bad background kind");
    const bool skybox = s->background_kind == RT_BG_SKYBOX;
    if (skybox)
        for (const HostTexture& t : s->skybox)
            if (t.width == 0 || t.height == 0 || t.rgb.size() != static_cast<size_t>(t.width) * t.height * 3)
                return fail(c, RT_E_INVALID, "skybox face without texels");
    if (s->camera.kind != RT_CAMERA_SIMPLE && s->camera.kind != RT_CAMERA_DOF)
        return fail(c, RT_E_INVALID, "bad camera kind");
    if (s->camera.kind == RT_CAMERA_DOF && s->camera.samples == 0)
        return fail(c, RT_E_INVALID, "DepthOfFieldCamera with 0 samples");
    bool needs_path = s->camera.kind == RT_CAMERA_DOF || skybox;
    std::vector<DevSphere> spheres;
    std::vector<double> sx, sy, sz, srad;
    std::vector<int32_t> sphere_obj, plane_obj;
    std::vector<DevPlane> planes;
    std::vector<DevMaterial> mats(s->objects.size());
    std::vector<DevLight> lights;
    for (size_t i = 0; i < s->objects.size(); ++i) {
        const rt_object& o = s->objects[i];
        if (o.material < RT_MAT_PHONG || o.material > RT_MAT_TRANSPARENT)
            return fail(c, RT_E_INVALID, "object " + std::to_string(i) + ": bad material kind");
        needs_path |= o.material == RT_MAT_INDIRECT_PHONG || o.material == RT_MAT_TRANSPARENT;
        if (o.shape == RT_SHAPE_SPHERE) {
            spheres.push_back(DevSphere{o.geom[0], o.geom[1], o.geom[2], o.geom[3] * o.geom[3]});
            sphere_obj.push_back(static_cast<int32_t>(i));
            sx.push_back(o.geom[0]); sy.push_back(o.geom[1]); sz.push_back(o.geom[2]); srad.push_back(o.geom[3]);
        } else if (o.shape == RT_SHAPE_PLANE) {
            planes.push_back(DevPlane{o.geom[0], o.geom[1], o.geom[2], o.geom[3], o.geom[4], o.geom[5]});
            plane_obj.push_back(static_cast<int32_t>(i));
        } else {
            return fail(c, RT_E_INVALID, "object " + std::to_string(i) + ": bad shape kind");
        }
        DevMaterial& m = mats[i];
        std::memset(&m, 0, sizeof m);
        const rt_color* src[3] = {&o.diffuse, &o.specular, &o.ambient};
        double* dst[3] = {m.kd, m.ks, m.amb};
        for (int k = 0; k < 3; ++k) { dst[k][0] = src[k]->r; dst[k][1] = src[k]->g; dst[k][2] = src[k]->b; }
        m.exponent = o.exponent;
        m.kd_sig = significance(o.diffuse);
        m.ks_sig = significance(o.specular);
        m.ior = o.ior;
        m.kind = o.material;
        m.samples = o.material == RT_MAT_INDIRECT_PHONG ? o.samples : 0;
    }
    for (size_t i = 0; i < s->lights.size(); ++i) {
        const rt_light& l = s->lights[i];
        if (l.kind < RT_LIGHT_POINT || l.kind > RT_LIGHT_AREA)
            return fail(c, RT_E_INVALID, "light " + std::to_string(i) + ": bad light kind");
        needs_path |= l.kind == RT_LIGHT_AREA;
        DevLight d{};
        for (int k = 0; k < 9; ++k) d.v[k] = l.v[k];
        d.color[0] = l.color.r; d.color[1] = l.color.g; d.color[2] = l.color.b;
        d.kind = l.kind;
        lights.push_back(d);
    }
    // Sphere BVH; spheres (and their object ids) are stored in its leaf order.
    // Box padding scales with the largest sphere-box coordinate (BVH exactness).
    double extent = 0.0;
    for (size_t k = 0; k < spheres.size(); ++k) {
        const double r = std::fabs(srad[k]);
        for (double v : {sx[k] - r, sx[k] + r, sy[k] - r, sy[k] + r, sz[k] - r, sz[k] + r})
            if (std::isfinite(v)) extent = std::max(extent, std::fabs(v));
    }
    // Leaves of 2 spheres measured fastest at C3; 4 when that tree and the
    // spheres would not fit the traversal kernels' LDS budget (tuning "bvh_leaf" overrides).
    const double pad = 1e-5 * (1.0 + extent);
    const int leaf_env = static_cast<int>(c->t(kTuneBvhLeaf));
    BvhResult bvh = build_sphere_bvh(sx, sy, sz, srad, pad, leaf_env > 0 ? leaf_env : 2);
    // leaves of 2 whatever the tree's size (C4 49.4 vs 50.3 ms, C5 293.3 vs 297.1 ms with 4 on one
    // box); 4 only for the quantised tree (tuning qtree), whose C4 tree then fits the LDS
    if (leaf_env <= 0 && c->t(kTuneQTree) != 0 &&
        bvh.nodes.size() * sizeof(DevBvhNode) + spheres.size() * (sizeof(DevSphere) + 4) > kLdsBudget)
        bvh = build_sphere_bvh(sx, sy, sz, srad, pad, 4);
    const Bvh4Result bvh4 = collapse_bvh4(bvh);
    // traversal stacks hold 64 entries (trace_common.hpp kBvhStack / kBvh4Stack)
    if (bvh_depth(bvh) > 64) return fail(c, RT_E_UNSUPPORTED, "sphere BVH deeper than the traversal stack");
    c->deep_bvh4 = bvh4_stack_need(bvh4) > 64;
    // compact stack (trace_common.hpp kShortStack, stk_entry16): the stack never holds more
    // entries than the deepest inner node's depth; node indices and leaf codes
    // (first << 3 | count - 1) must fit a signed 16-bit field; the whole-LDS walk stores inner
    // nodes as byte offsets (c + 1) * 8 (trace_common.hpp node_byte_off)
    c->short_stack = bvh_depth(bvh) <= 32 && bvh.nodes.size() < 4095 && spheres.size() <= 4096;
    c->short_stack18 = bvh_depth(bvh) <= 32 && bvh.nodes.size() < 131072 && spheres.size() <= 16383;
    // binary16 nodes only for trees that do not fit LDS whole (the prefix source reads them)
    const bool big_tree = bvh.nodes.size() * sizeof(DevBvhNode) + spheres.size() * (sizeof(DevSphere) + 4) > kLdsBudget;
    const std::vector<DevBvhNodeH> hnodes = big_tree ? half_nodes(bvh) : std::vector<DevBvhNodeH>{};
    // the quantised 4-wide tree (nearest_q4's stack holds kQ4Stack entries), for every tree
    // (tuning qtree, or src 25 / 26, select it)
    const std::vector<DevQNode4> qnodes = bvh4_stack_need(bvh4) <= kQ4Stack ? quantize_bvh4(bvh4) : std::vector<DevQNode4>{};
    std::vector<double> r_leaf(spheres.size());
    {
        std::vector<DevSphere> s2(spheres.size());
        std::vector<int32_t> o2(spheres.size());
        for (size_t k = 0; k < spheres.size(); ++k) {
            s2[k] = spheres[bvh.order[k]]; o2[k] = sphere_obj[bvh.order[k]]; r_leaf[k] = srad[bvh.order[k]];
        }
        spheres.swap(s2);
        sphere_obj.swap(o2);
    }
    // light-view grids of the point lights (tuning: "light_grids" 0 disables, "light_grid_res" forces the resolution)
    LightGridResult lg;
    if (c->t(kTuneLgrid) != 0) lg = build_light_grids(spheres, r_leaf, lights, pad, static_cast<int>(c->t(kTuneLgridRes)));
    // the camera's view grid (generation 0, tuning "cam" 3): a cell about 8 x 8 pixels of the
    // scene's own frame size, im_dist * max(W, H) / 8 cells per face side (tuning "cam_grid_res");
    // only for scenes the wavefront schedule can render (the path kernel never reads it)
    LightGridResult cg;
    if (s->camera.kind == RT_CAMERA_SIMPLE && !needs_path && c->t(kTuneCamGridRes) >= 0)
        cg = build_view_grid(spheres, r_leaf, s->camera.position, pad, view_grid_res(s, c->t(kTuneCamGridRes)),
                             view_grid_cap(spheres.size()));
    // One blob: [spheres][sphere_obj][planes][plane_obj][mats][lights][bvh], 256-B aligned pieces.
    size_t off = 0;
    auto place = [&](size_t bytes) { size_t at = off; off = align_up(off + bytes, 256); return at; };
    const size_t o_sph = place(spheres.size() * sizeof(DevSphere));
    const size_t o_sobj = place(sphere_obj.size() * sizeof(int32_t));
    const size_t o_pl = place(planes.size() * sizeof(DevPlane));
    const size_t o_pobj = place(plane_obj.size() * sizeof(int32_t));
    const size_t o_mat = place(mats.size() * sizeof(DevMaterial));
    const size_t o_li = place(lights.size() * sizeof(DevLight));
    const size_t o_bvh = place(bvh.nodes.size() * sizeof(DevBvhNode));
    const size_t o_bvh4 = place(bvh4.planes.size() * sizeof(DevBvh4Plane));
    const size_t o_bvhh = place(hnodes.size() * sizeof(DevBvhNodeH));
    const size_t o_q4 = place(qnodes.size() * sizeof(DevQNode4));
    const size_t o_srgbv = place(256 * sizeof(double));
    const size_t o_lg = place(lg.grids.size() * sizeof(DevLightGrid));
    const size_t o_lgoff = place(lg.off.size() * sizeof(uint32_t));
    const size_t o_lgent = place(lg.ent.size() * sizeof(DevLgEntry));
    const size_t o_cg = place(cg.grids.size() * sizeof(DevLightGrid));
    const size_t o_cgoff = place(cg.off.size() * sizeof(uint32_t));
    const size_t o_cgent = place(cg.ent.size() * sizeof(DevLgEntry));
    size_t tex_bytes = 0;
    uint64_t face_off[6] = {0, 0, 0, 0, 0, 0};
    if (skybox)
        for (int k = 0; k < 6; ++k) { face_off[k] = tex_bytes; tex_bytes += s->skybox[k].rgb.size(); }
    const size_t o_tex = place(tex_bytes);
    const size_t total = off ? off : 256;
    std::vector<uint8_t> host(total, 0);
    auto put = [&](size_t at, const void* p, size_t bytes) { if (bytes) std::memcpy(host.data() + at, p, bytes); };
    put(o_sph, spheres.data(), spheres.size() * sizeof(DevSphere));
    put(o_sobj, sphere_obj.data(), sphere_obj.size() * sizeof(int32_t));
    put(o_pl, planes.data(), planes.size() * sizeof(DevPlane));
    put(o_pobj, plane_obj.data(), plane_obj.size() * sizeof(int32_t));
    put(o_mat, mats.data(), mats.size() * sizeof(DevMaterial));
    put(o_li, lights.data(), lights.size() * sizeof(DevLight));
    put(o_bvh, bvh.nodes.data(), bvh.nodes.size() * sizeof(DevBvhNode));
    put(o_bvh4, bvh4.planes.data(), bvh4.planes.size() * sizeof(DevBvh4Plane));
    put(o_bvhh, hnodes.data(), hnodes.size() * sizeof(DevBvhNodeH));
    put(o_q4, qnodes.data(), qnodes.size() * sizeof(DevQNode4));
    put(o_srgbv, srgb_values_table(), 256 * sizeof(double));
    put(o_lg, lg.grids.data(), lg.grids.size() * sizeof(DevLightGrid));
    put(o_lgoff, lg.off.data(), lg.off.size() * sizeof(uint32_t));
    put(o_lgent, lg.ent.data(), lg.ent.size() * sizeof(DevLgEntry));
    put(o_cg, cg.grids.data(), cg.grids.size() * sizeof(DevLightGrid));
    put(o_cgoff, cg.off.data(), cg.off.size() * sizeof(uint32_t));
    put(o_cgent, cg.ent.data(), cg.ent.size() * sizeof(DevLgEntry));
    if (skybox)
        for (int k = 0; k < 6; ++k) put(o_tex + face_off[k], s->skybox[k].rgb.data(), s->skybox[k].rgb.size());
    // every render still reading the old blob (on any stream) must be done before it is overwritten
    if (c->render_pending) HIP_TRY(c, hipEventSynchronize(c->render_done));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (c->d_blob && c->blob_bytes < total) { (void)hipFree(c->d_blob); c->d_blob = nullptr; c->blob_bytes = 0; }
    if (!c->d_blob) {
        HIP_TRY(c, hipMalloc(&c->d_blob, total));
        c->blob_bytes = total;
    }
    HIP_TRY(c, hipMemcpy(c->d_blob, host.data(), total, hipMemcpyHostToDevice));
    auto* base = static_cast<uint8_t*>(c->d_blob);
    DevScene& d = c->dsc;
    d = DevScene{};
    d.spheres = reinterpret_cast<const DevSphere*>(base + o_sph);
    d.sphere_obj = reinterpret_cast<const int32_t*>(base + o_sobj);
    d.planes = reinterpret_cast<const DevPlane*>(base + o_pl);
    d.plane_obj = reinterpret_cast<const int32_t*>(base + o_pobj);
    d.mats = reinterpret_cast<const DevMaterial*>(base + o_mat);
    d.lights = reinterpret_cast<const DevLight*>(base + o_li);
    d.bvh = reinterpret_cast<const DevBvhNode*>(base + o_bvh);
    d.bvh_root = bvh.root;
    d.n_spheres = static_cast<int32_t>(spheres.size());
    d.n_planes = static_cast<int32_t>(planes.size());
    d.n_lights = static_cast<int32_t>(lights.size());
    d.n_bvh = static_cast<int32_t>(bvh.nodes.size());
    d.bvh4 = reinterpret_cast<const DevBvh4Plane*>(base + o_bvh4);
    d.bvh4_root = bvh4.root;
    d.n_bvh4 = bvh4.n_nodes;
    d.bvh_h = hnodes.empty() ? nullptr : reinterpret_cast<const DevBvhNodeH*>(base + o_bvhh);
    d.q4 = qnodes.empty() ? nullptr : reinterpret_cast<const DevQNode4*>(base + o_q4);
    d.n_q4 = static_cast<int32_t>(qnodes.size());
    c->q4_ok = !qnodes.empty();
    d.has_fresnel = 0;
    for (const DevMaterial& m : mats) d.has_fresnel |= m.kind == kMatFresnel ? 1 : 0;
    d.needs_path = needs_path ? 1 : 0;
    d.skybox = skybox ? 1 : 0;
    d.tex = base + o_tex;
    d.srgb_values = reinterpret_cast<const double*>(base + o_srgbv);
    for (int k = 0; k < 6; ++k)
        d.faces[k] = DevTexFace{skybox ? s->skybox[k].width : 0u, skybox ? s->skybox[k].height : 0u, face_off[k]};
    d.cam_dof = s->camera.kind == RT_CAMERA_DOF ? 1 : 0;
    d.cam_samples = d.cam_dof ? s->camera.samples : 1u;
    d.cam_focus = s->camera.focus;
    d.cam_aperture = s->camera.aperture;
    {   // camera.rs:98: im_dist = (matrix * Vec3(0, 0, 1)).norm()
        const double* M = s->camera.matrix;
        const double zx = (M[0] * 0.0 + M[1] * 0.0) + M[2] * 1.0;
        const double zy = (M[3] * 0.0 + M[4] * 0.0) + M[5] * 1.0;
        const double zz = (M[6] * 0.0 + M[7] * 0.0) + M[8] * 1.0;
        d.cam_im_dist = std::sqrt(zx * zx + zy * zy + zz * zz);
    }
    for (int k = 0; k < 3; ++k) d.cam_pos[k] = s->camera.position[k];
    for (int k = 0; k < 9; ++k) d.cam_m[k] = s->camera.matrix[k];
    d.bg[0] = s->background.r; d.bg[1] = s->background.g; d.bg[2] = s->background.b;
    d.lgrid = lg.grids.empty() ? nullptr : reinterpret_cast<const DevLightGrid*>(base + o_lg);
    d.lg_off = reinterpret_cast<const uint32_t*>(base + o_lgoff);
    d.lg_ent = reinterpret_cast<const DevLgEntry*>(base + o_lgent);
    d.cgrid = (cg.grids.empty() || cg.grids[0].R <= 0) ? nullptr : reinterpret_cast<const DevLightGrid*>(base + o_cg);
    d.cg_off = reinterpret_cast<const uint32_t*>(base + o_cgoff);
    d.cg_ent = reinterpret_cast<const DevLgEntry*>(base + o_cgent);
    c->all_lights_gridded = !lights.empty() && lg.grids.size() == lights.size();
    for (const DevLightGrid& g : lg.grids) c->all_lights_gridded = c->all_lights_gridded && g.R > 0;
    c->scene_spp = s->antialias;
    c->has_scene = true;
    return RT_OK;
}

int rt_scene_upload(rt_ctx* c, const rt_scene* s) {
    if (!c || !s) return RT_E_INVALID;
    return guarded(c, [&] { return scene_upload(c, s); });
}

static int check_opts(rt_ctx* c, const rt_render_opts* o, uint32_t& spp, uint32_t& band, uint32_t& stride, uint32_t& pitch) {
    if (!o) return fail(c, RT_E_INVALID, "null opts");
    if (o->width == 0 || o->height == 0) return fail(c, RT_E_INVALID, "empty frame");
    if (o->jitter != RT_JITTER_CENTER && o->jitter != RT_JITTER_RANDOM) return fail(c, RT_E_INVALID, "bad jitter mode");
    if (o->max_depth > RT_MAX_DEPTH_LIMIT) return fail(c, RT_E_INVALID, "max_depth above RT_MAX_DEPTH_LIMIT");
    band = o->band ? o->band : 1;
    stride = o->band_stride ? o->band_stride : 1;
    if (o->band_phase >= stride) return fail(c, RT_E_INVALID, "band_phase >= band_stride");
    if (static_cast<uint64_t>(o->x0) + o->tile_w > o->width) return fail(c, RT_E_INVALID, "tile exceeds frame width");
    if (o->tile_h) {
        uint64_t j = o->tile_h - 1;
        uint64_t last = o->y0 + ((j / band) * stride + o->band_phase) * band + j % band;
        if (last >= o->height) return fail(c, RT_E_INVALID, "tile exceeds frame height");
    }
    spp = o->spp ? o->spp : c->scene_spp;                     // 0: the scene's Options.antialias
    if (spp == 0) return fail(c, RT_E_INVALID, "spp is 0 and the scene's antialias is 0");
    pitch = o->bgr_pitch ? o->bgr_pitch : 3 * o->tile_w;
    if (pitch < 3 * o->tile_w) return fail(c, RT_E_INVALID, "bgr_pitch < 3*tile_w");
    if (o->algo < RT_ALGO_AUTO || o->algo > RT_ALGO_PATH) return fail(c, RT_E_INVALID, "bad algo");
    return RT_OK;
}

// The stream of rt_render's device -> host copies.  A CU-masked stream (mask = every CU) gets a
// hardware queue of its own (ensure_bstreams), so the copies never queue behind the render's launches.
static int ensure_copy_stream(rt_ctx* c) {
    if (c->copy_stream) return RT_OK;
    std::vector<uint32_t> mask((c->n_cu + 31) / 32, 0u);
    for (int cu = 0; cu < c->n_cu; ++cu) mask[cu / 32] |= 1u << (cu % 32);
    if (hipExtStreamCreateWithCUMask(&c->copy_stream, static_cast<uint32_t>(mask.size()), mask.data()) != hipSuccess) {
        (void)hipGetLastError();
        HIP_TRY(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    }
    return RT_OK;
}

// Device buffers of the sparse host copies for a tw x rows tile (segment bits, row counts, row
// offsets, and the packed BGR / RGB sections of the outputs requested at their largest: every
// segment flagged), grown on demand.  They are not part of the working-set budget, so they are
// taken only from what the device has free beyond kRuntimeHeadroom; if they do not fit (or
// hipMalloc fails) *ok is false and the render copies its frame the plain way.
static int ensure_sparse(rt_ctx* c, hipStream_t st, uint32_t tw, uint32_t rows, bool bgr, bool rgb, bool* ok) {
    *ok = false;
    int rc = ensure_copy_stream(c);
    if (rc != RT_OK) return rc;
    if (!c->sp_cam) HIP_TRY(c, hipEventCreateWithFlags(&c->sp_cam, hipEventDisableTiming));
    if (!c->sp_ready) HIP_TRY(c, hipEventCreateWithFlags(&c->sp_ready, hipEventDisableTiming));
    const uint64_t nseg = (tw + kSegPx - 1) / kSegPx, words = (nseg + 31) / 32, segs = nseg * rows;
    const uint64_t s_bits = align_up(rows * words * 4, 256), s_cnt = align_up(rows * 4ull, 256),
                   s_off = align_up((rows + 1ull) * 4, 256), s_bgr = bgr ? align_up(segs * 3 * kSegPx, 256) : 0,
                   s_rgb = rgb ? segs * 3 * kSegPx * sizeof(float) : 0;
    const uint64_t need = s_bits + s_cnt + s_off + s_bgr + s_rgb;
    if (need > c->sp_cap) {
        HIP_TRY(c, hipStreamSynchronize(st));
        HIP_TRY(c, hipStreamSynchronize(c->copy_stream));
        if (c->d_sp) (void)hipFree(c->d_sp);
        c->d_sp = nullptr;
        c->sp_cap = 0;
        size_t fr = 0, total = 0;
        if (hipMemGetInfo(&fr, &total) != hipSuccess) { (void)hipGetLastError(); return RT_OK; }
        if (need > fr || fr - need < kRuntimeHeadroom) return RT_OK;
        if (hipMalloc(&c->d_sp, need) != hipSuccess) {
            (void)hipGetLastError();
            c->d_sp = nullptr;
            return RT_OK;
        }
        c->sp_cap = need;
    }
    auto* base = static_cast<uint8_t*>(c->d_sp);
    c->d_sp_bits = reinterpret_cast<uint32_t*>(base);
    c->d_sp_cnt = reinterpret_cast<uint32_t*>(base + s_bits);
    c->d_sp_off = reinterpret_cast<uint32_t*>(base + s_bits + s_cnt);
    c->d_sp_bgr = bgr ? base + s_bits + s_cnt + s_off : nullptr;
    c->d_sp_rgb = rgb ? reinterpret_cast<float*>(base + s_bits + s_cnt + s_off + s_bgr) : nullptr;
    *ok = true;
    return RT_OK;
}

// rt_ctx_reserve: a no-op launch with private memory on every stream of the schedule (the
// code objects load, each hardware queue and its scratch are set up), then wait for them.
static int warm_streams(rt_ctx* c, const std::vector<hipStream_t>& ss) {
    for (hipStream_t s : ss) {
        if (!s) continue;
        HIP_TRY(c, launch_warmup(static_cast<uint32_t>(2 * c->n_cu), s));
        HIP_TRY(c, launch_path_warmup(s));
    }
    for (hipStream_t s : ss)
        if (s) HIP_TRY(c, hipStreamSynchronize(s));
    return RT_OK;
}

// dry (rt_ctx_reserve): every allocation and stream the render would make, then warm_streams
// instead of the launches; counters and the last render's statistics are left alone.
static int render_device(rt_ctx* c, const rt_render_opts* o, void* d_rgb, void* d_bgr, void* stream, bool dry = false) {
    if (!c->has_scene) return fail(c, RT_E_NOSCENE, "no scene uploaded");
    uint32_t spp, band, stride, pitch;
    int rc = check_opts(c, o, spp, band, stride, pitch);
    if (rc != RT_OK) return rc;
    if (o->flags & RT_OUT_FRAME_ROWS) return fail(c, RT_E_INVALID, "RT_OUT_FRAME_ROWS is for rt_render's host buffers");
    HIP_TRY(c, hipSetDevice(c->device));
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : c->stream;
    // The context's working sets (counters, wavefront buffers, path stacks) are
    // shared by its renders: a render on another stream waits for the previous one.
    // (on the stream the previous render ended on, stream order alone suffices)
    if (c->render_pending && st != c->done_stream) HIP_TRY(c, hipStreamWaitEvent(st, c->render_done, 0));
    FrameParams fp{};
    fp.hw = static_cast<double>(o->width) / 2.0;              // main.rs:39-41
    fp.hh = static_cast<double>(o->height) / 2.0;
    fp.scale = std::fmax(1.0 / fp.hw, 1.0 / fp.hh);
    fp.x0 = o->x0; fp.tile_w = o->tile_w; fp.y0 = o->y0; fp.tile_h = o->tile_h;
    fp.band = band; fp.band_stride = stride; fp.band_phase = o->band_phase;
    fp.max_depth = o->max_depth;
    fp.spp = spp;
    fp.bgr_pitch = pitch;
    fp.out_rgb = (o->flags & RT_OUT_RGB_F32) ? static_cast<float*>(d_rgb) : nullptr;
    fp.out_bgr = (o->flags & RT_OUT_BGR_U8) ? static_cast<uint8_t*>(d_bgr) : nullptr;
    fp.counters = c->d_counters;
    fp.jitter = o->jitter;
    fp.seed = o->seed;
    fp.srgb = c->d_srgb;
    {
        // The background pixel exactly as average_samples + to_srgb produce it on the
        // device (same f64 operations): camera misses are written by wf_nearest directly.
        double px[3];
        for (int k = 0; k < 3; ++k) {
            const double cam = (0.0 + c->dsc.bg[k]) / 1.0;        // raytrace.rs:270-276, one camera sample
            double acc = 0.0;
            for (uint32_t q = 0; q < spp; ++q) acc = acc + cam;    // main.rs:47-55
            px[k] = acc / static_cast<double>(spp);
            fp.bg_rgb[k] = static_cast<float>(px[k]);
        }
        fp.bg_bgr[0] = to_srgb(px[2]);                             // color.rs:628-632, B G R
        fp.bg_bgr[1] = to_srgb(px[1]);
        fp.bg_bgr[2] = to_srgb(px[0]);
    }
    fp.row0 = 0;
    fp.rows = o->tile_h;
    const size_t lds_bytes = static_cast<size_t>(c->dsc.n_spheres) * sizeof(DevSphere);
    const bool fits_lds = lds_bytes <= 64 * 1024;
    int mode = o->algo;
    // the stochastic / branching classes, and random jitter with several AA
    // samples per pixel, run on the path kernel only (the chain schedules trace
    // one camera ray per pixel: centre jitter, or random jitter with spp = 1)
    const bool path_only = c->dsc.needs_path || (o->jitter != RT_JITTER_CENTER && spp > 1);
    if (mode == RT_ALGO_AUTO)
        mode = path_only ? RT_ALGO_PATH
                         : (c->dsc.n_lights <= 32 ? RT_ALGO_WAVEFRONT : (fits_lds ? RT_ALGO_BRUTE_LDS : RT_ALGO_BRUTE_GLOBAL));
    if (path_only && mode != RT_ALGO_PATH)
        return fail(c, RT_E_UNSUPPORTED,
                    "IndirectPhong / Transparent materials, AreaLight, DepthOfFieldCamera and random jitter with "
                    "spp > 1 need RT_ALGO_PATH");
    if (mode == RT_ALGO_BRUTE_LDS && lds_bytes > 160 * 1024)
        return fail(c, RT_E_INVALID, "sphere list does not fit in LDS; use RT_ALGO_BRUTE_GLOBAL");
    if ((mode == RT_ALGO_WAVEFRONT || mode == RT_ALGO_WAVEFRONT_BRUTE) && c->dsc.n_lights > 32)
        return fail(c, RT_E_UNSUPPORTED, "the wavefront path handles at most 32 lights");
    // the statistics counters start at zero: cleared here, or, for a one-chunk wavefront render
    // without RT_COUNT_WORK (its tally is lazy), by flush_tally just before that tally
    auto zero_counters = [&]() -> int {
        HIP_TRY(c, hipMemsetAsync(c->d_counters, 0, kCounterWords * sizeof(unsigned long long), st));
        return RT_OK;
    };
    if (!dry) {
        c->tally.on = false;
        c->last_pixels = static_cast<uint64_t>(o->tile_w) * o->tile_h;
        c->last_stream = st;
        c->last_spp_traced = 1;
        c->last_chunks = 0;
    }
    c->n_bands = 0;
    c->sparse_on = false;
    if (dry && (o->tile_w == 0 || o->tile_h == 0)) return warm_streams(c, {st});
    if (o->tile_w == 0 || o->tile_h == 0) {
        if ((rc = zero_counters()) != RT_OK) return rc;
        c->last_timed = false;
        HIP_TRY(c, hipEventRecord(c->render_done, st));
        c->done_stream = st;
        c->render_pending = true;
        return RT_OK;
    }
    if (mode == RT_ALGO_WAVEFRONT || mode == RT_ALGO_WAVEFRONT_BRUTE) {
        // LDS per traversal workgroup (1024 threads, two resident per CU): the
        // whole BVH + sphere list when they fit, else the top of the tree.
        const size_t node_bytes = static_cast<size_t>(c->dsc.n_bvh) * sizeof(DevBvhNode);
        const size_t sph_bytes = static_cast<size_t>(c->dsc.n_spheres) * (sizeof(DevSphere) + sizeof(int32_t));
        const size_t node4_bytes = static_cast<size_t>(c->dsc.n_bvh4) * kBvh4Planes * sizeof(DevBvh4Plane);
        // (nearest, occlusion) sphere sources, see launch_api.hpp.  Default: the
        // binary tree for the nearest-hit query and the 4-wide tree for the
        // shadow query, each staged whole in LDS with the spheres when it fits
        // (measured best at C3); tuning "src" / "src_occ" override.
        int src, src_occ;
        if (mode == RT_ALGO_WAVEFRONT) {
            const bool fit2 = node_bytes + sph_bytes <= kLdsBudget;
            const bool fit4 = node4_bytes + sph_bytes <= kLdsBudget;
            const bool q4_fits = static_cast<size_t>(c->dsc.n_q4) * sizeof(DevQNode4) <= kLdsBudget;
            const bool compact = c->t(kTuneCompact) != 0;
            // is (nearest, shadow) source pair (a, o) available for this scene (launch_wavefront's pairs)?
            auto pair_ok = [&](int a, int o) {
                if (c->deep_bvh4) return (a == 7 && o == 7 && fit2) || (a == 2 && o == 2);   // the 4-wide stack could overflow
                switch (a * 100 + o) {
                case 202: case 211: return true;
                case 707: case 710: return fit2 && (o == 7 || fit4);
                case 910: return fit2 && fit4 && c->short_stack;
                case 511: return c->dsc.bvh_h != nullptr;
                case 611: return c->dsc.bvh_h != nullptr && c->short_stack18;
                case 811: return true;
                case 2511: return c->q4_ok && q4_fits;
                case 2611: return c->q4_ok;
                default: return false;
                }
            };
            // Default: both trees whole in LDS with the spheres (measured best at C3), the binary
            // tree for the nearest hit (compact stack entries where the tree allows) and the 4-wide
            // tree for shadow rays without a light grid; trees beyond LDS: the binary tree's
            // breadth-first top in LDS (binary16 bounds where representable, twice the nodes)
            // and the 4-wide shadow tree through L2; the quantised tree with tuning "qtree".
            if (fit2 && fit4) {
                src = c->short_stack && compact ? 9 : 7;
                src_occ = 10;
            } else {
                src = !c->dsc.bvh_h || c->t(kTuneHalf) == 0 ? 8 : c->short_stack18 && compact ? 6 : 5;
                src_occ = 11;
                if (c->q4_ok && c->t(kTuneQTree) != 0) src = q4_fits ? 25 : 26;
            }
            if (c->deep_bvh4) src_occ = src = fit2 ? 7 : 2;
            if (c->t(kTuneSrc) >= 0) {                   // forced (A/B measurement, tests)
                src = static_cast<int>(c->t(kTuneSrc));
                src_occ = c->t(kTuneSrcOcc) >= 0 ? static_cast<int>(c->t(kTuneSrcOcc)) : src;
            }
            if (!pair_ok(src, src_occ)) {               // unsupported or unavailable here: the binary tree through L2
                src = 2;
                src_occ = c->deep_bvh4 ? 2 : 11;
            }
            // LDS prefix (tuning "prefix_kb"): measured at C4, 64 KB of binary nodes for the nearest-hit kernels
            const int kb2 = static_cast<int>(c->t(kTunePrefixKb2));
            c->dsc.pfx2 = static_cast<int32_t>(static_cast<size_t>(std::max(kb2, 1)) * 1024 / sizeof(DevBvhNode));
            c->dsc.pfxq = static_cast<int32_t>(static_cast<size_t>(std::max(kb2, 1)) * 1024 / sizeof(DevQNode4));
        } else {
            src = src_occ = fits_lds ? 1 : 0;
        }
        // tuning "split" 0: every kernel on one in-order stream (A/B measurement);
        // "deal": 1 workgroup-major chunk dealing (default), 0 workgroup-first;
        // "bstreams": streams for the shadow + shading kernels (default 2;
        // generations alternate over them).
        // default: two B streams when the tree is in LDS (C3: 3.30 vs 3.71 ms on one stream);
        // one stream when the nearest-hit walk reads the tree through L2 below its LDS prefix,
        // where the overlapped shadow / shading waves slow that chain more than they hide
        // (C4 55.2 vs 56.6-57.3 ms, C5 318 vs 330 ms, binary16 nodes; round 5 with the
        // high-priority chain: C4 51.9 vs 50.4 ms)
        const bool prefix_src = src == 5 || src == 6 || src == 8 || src == 26;
        const bool split = c->t(kTuneSplit) < 0 ? !prefix_src : c->t(kTuneSplit) != 0;
        // two b streams (consecutive generations' shadows and shading overlap): measured
        // 3.87 -> 3.78 ms at C3 once the shading runs in its own kernel; three are slower
        const int n_b = std::max(1, std::min(kMaxBStreams, static_cast<int>(c->t(kTuneBStreams))));
        // generation 0: the camera's view grid (any sphere source), spheres staged in LDS when they
        // fit (3), else through L2 (4); the default where built (C3 camera pass 520 -> 327 us, 3.46 ->
        // 3.26 ms per frame on one box, against the camera-view tile walk it replaced); otherwise
        // (tuning "cam" other than 3 or -1, or no grid) per ray through the nearest-hit source
        int cam = 0;
        if ((c->t(kTuneCam) == 3 || (c->t(kTuneCam) < 0 && mode == RT_ALGO_WAVEFRONT)) && c->dsc.cgrid)
            cam = static_cast<size_t>(c->dsc.n_spheres) * (sizeof(DevSphere) + sizeof(int32_t)) <= kLdsBudget ? 3 : 4;
        const uint32_t wg_major = c->t(kTuneDeal) != 0 ? 1u : 0u;
        if (c->t(kTuneVerbose))
            std::fprintf(stderr, "rtamd: wavefront src %d occ %d cam %d deep4 %d short_stack %d split %d pfx %d/%d\n",
                         src, src_occ, cam, c->deep_bvh4 ? 1 : 0, c->short_stack ? 1 : 0, split ? 1 : 0, c->dsc.pfx2,
                         c->dsc.pfxq);
        // Chunks of whole rows, multiples of 8 (the generation-0 8x8 tiles), sized so
        // the lanes' working sets (ensure_wf: queues, one shade-record array and one
        // level array per lit generation, terminals) fit the budget:
        // tuning "wf_budget_mb", else min(80 GB, 85% of the free device memory)
        // (hipMemGetInfo), e.g. C4's 8192^2 frame in one chunk at depth 8 (62.8 vs
        // 63.9 ms as two) and C5 in 7 at depth 16.  Balanced: a frame slightly over
        // the cap becomes two halves, not a full chunk plus a sliver that pays every
        // generation's launch latency again.  If hipMalloc still runs out of memory
        // (another context, a caller's buffers), the chunks are halved and the
        // allocation retried; results do not depend on the chunking.
        const uint64_t levels = o->max_depth + 1ull;
        const int lanes_req = static_cast<int>(c->t(kTuneLanes));
        uint64_t cap_px = static_cast<uint64_t>(c->t(kTuneChunkPixels));
        if (cap_px == 0) {
            const uint64_t budget = c->t(kTuneWfBudgetMb) > 0 ? static_cast<uint64_t>(c->t(kTuneWfBudgetMb)) << 20
                                                               : default_wf_budget(c);
            cap_px = std::max<uint64_t>(1, budget / static_cast<uint64_t>(lanes_req) / wf_bytes_per_slot(levels));
        }
        // rt_render into host memory: chunks of at most tile_h / host_chunks rows (the copy of a
        // chunk's rows overlaps the later chunks' generations); host_first sizes the first of two
        uint32_t first_rows = 0;
        if (c->want_bands && c->t(kTuneHostChunks) > 1) {
            const uint64_t hc = static_cast<uint64_t>(c->t(kTuneHostChunks));
            const uint64_t pf = static_cast<uint64_t>(c->t(kTuneHostFirst));
            if (hc == 2 && pf > 0) {
                first_rows = static_cast<uint32_t>(std::max<uint64_t>(8, (o->tile_h * pf / 100) / 8 * 8));
                if (first_rows >= o->tile_h) first_rows = 0;
                else cap_px = std::min<uint64_t>(cap_px, static_cast<uint64_t>((std::max(first_rows, o->tile_h - first_rows) + 7) / 8 * 8) * o->tile_w);
            }
            if (first_rows == 0) cap_px = std::min<uint64_t>(cap_px, ((o->tile_h + hc - 1) / hc + 7) / 8 * 8 * o->tile_w);
        }
        const uint32_t tiles_x = (o->tile_w + 7) / 8;
        const int mark_gen = std::max(0, std::min<int>(static_cast<int>(c->t(kTuneStaggerGen)), static_cast<int>(o->max_depth) + 1));
        uint32_t chunk_rows = 0, n_chunks = 0, G = 1, R = 0;
        int n_lanes = 1;
        for (;;) {
            chunk_rows = static_cast<uint32_t>(std::max<uint64_t>(8, std::min<uint64_t>(cap_px / o->tile_w, UINT32_MAX) / 8 * 8));
            chunk_rows = std::min(chunk_rows, (o->tile_h + 7) / 8 * 8);
            n_chunks = (o->tile_h + chunk_rows - 1) / chunk_rows;
            chunk_rows = std::max<uint32_t>(8, ((o->tile_h + n_chunks - 1) / n_chunks + 7) / 8 * 8);
            if (first_rows) {                      // two chunks of first_rows and tile_h - first_rows rows
                const uint32_t need = (std::max(first_rows, o->tile_h - first_rows) + 7) / 8 * 8;
                if (n_chunks == 2 && need * static_cast<uint64_t>(o->tile_w) <= cap_px) chunk_rows = need;
                else first_rows = 0;
            }
            n_lanes = std::max(1, std::min<int>(lanes_req, static_cast<int>(n_chunks)));
            int rc2 = ensure_lanes(c, n_lanes);
            if (rc2 != RT_OK) return rc2;
            const uint32_t slots = tiles_x * 64 * (chunk_rows / 8);
            const uint32_t cap = o->tile_w * chunk_rows;
            // G regions = workgroups per queue launch: two per CU, i.e. every
            // workgroup resident at once (1024 threads with the LDS-staged BVH),
            // so the wave-chunk dealing spreads even a small tail queue over the
            // whole chip in one round; fewer for small chunks; R covers every slot.
            const int g_env = static_cast<int>(c->t(kTuneRegions));
            G = g_env > 0 ? static_cast<uint32_t>(g_env) : 2u * static_cast<uint32_t>(c->n_cu);
            G = std::max<uint32_t>(1, std::min<uint32_t>({G, static_cast<uint32_t>(kMaxRegions), (slots + kWfThreads - 1) / kWfThreads}));
            R = (slots + G * kWfThreads - 1) / (G * kWfThreads) * kWfThreads;
            for (int l = 0; l < n_lanes && rc2 == RT_OK; ++l) {
                if (split && (rc2 = ensure_bstreams(c, c->lanes[l], n_b)) != RT_OK) return rc2;
                rc2 = ensure_wf(c, c->lanes[l], cap, G, R, static_cast<uint32_t>(levels));
            }
            if (rc2 == RT_OK) break;
            if (rc2 != RT_E_NOMEM || chunk_rows <= 8) return rc2;
            for (auto& L : c->lanes) drop_lane_memory(L);      // retry with half the pixels per chunk
            cap_px = std::max<uint64_t>(1, static_cast<uint64_t>(chunk_rows) * o->tile_w / 2);
        }
        // sparse host copies: a whole tile (contiguous rows or row bands) in one chunk on one lane,
        // pixels written where they end
        c->sparse_on = c->want_sparse && n_chunks == 1 && n_lanes == 1 && c->t(kTuneCompose) == 0 &&
                       (fp.out_rgb || fp.out_bgr);
        if (c->sparse_on) {
            bool ok = false;
            if ((rc = ensure_sparse(c, st, o->tile_w, o->tile_h, fp.out_bgr != nullptr, fp.out_rgb != nullptr, &ok)) != RT_OK)
                return rc;
            if (!ok && c->t(kTuneVerbose)) std::fprintf(stderr, "rtamd: sparse copy buffers do not fit: plain copies\n");
            c->sparse_on = ok;
        }
        if (dry) {
            std::vector<hipStream_t> ss{st};
            if (c->want_bands) {                   // rt_render's copy stream and its band events
                if ((rc = ensure_copy_stream(c)) != RT_OK) return rc;
                ss.push_back(c->copy_stream);
                for (uint32_t i = 0; i < n_chunks && i < static_cast<uint32_t>(kMaxBands); ++i)
                    if (!c->band_ev[i]) HIP_TRY(c, hipEventCreateWithFlags(&c->band_ev[i], hipEventDisableTiming));
            }
            for (int l = 0; l < n_lanes; ++l) {
                ss.push_back(c->lanes[l].s);
                if (split)
                    for (int i = 0; i < n_b; ++i) ss.push_back(c->lanes[l].sb[i]);
            }
            return warm_streams(c, ss);
        }
        for (int l = 0; l < n_lanes; ++l) {
            c->lanes[l].b.tiles_x = tiles_x;
            c->lanes[l].b.wg_major = wg_major;
            c->lanes[l].b.spread_below = static_cast<uint32_t>(c->t(kTuneSpreadBelow));
            c->lanes[l].b.compose = c->t(kTuneCompose) != 0 ? 1u : 0u;
            c->lanes[l].b.mark = c->sparse_on ? 1u : 0u;
        }
        c->last_chunks = n_chunks;
        auto chunk_row0 = [&](uint32_t ci) { return first_rows ? (ci ? first_rows : 0u) : ci * chunk_rows; };
        auto chunk_nrows = [&](uint32_t ci) {
            return first_rows ? (ci ? o->tile_h - first_rows : first_rows) : std::min(chunk_rows, o->tile_h - ci * chunk_rows);
        };
        // rt_render copies each chunk's rows as soon as that chunk's fold is done (the fold
        // runs in chain order, so a chunk's rows are final together)
        c->n_bands = 0;
        if (c->want_bands && n_chunks <= static_cast<uint32_t>(kMaxBands)) {
            for (uint32_t i = 0; i < n_chunks; ++i) {
                if (!c->band_ev[i]) HIP_TRY(c, hipEventCreateWithFlags(&c->band_ev[i], hipEventDisableTiming));
                c->band_row0[i] = chunk_row0(i);
                c->band_nrows[i] = chunk_nrows(i);
            }
            c->n_bands = static_cast<int>(n_chunks);
        }
        if (c->t(kTuneVerbose))
            std::fprintf(stderr, "rtamd: chunks %u x %u rows (first %u), lanes %d, G %u, R %u\n", n_chunks, chunk_rows, first_rows,
                         n_lanes, G, R);
        const bool count = (o->flags & RT_COUNT_WORK) != 0;
        const bool lazy_tally = n_chunks == 1 && n_lanes == 1;
        if ((!lazy_tally || count) && (rc = zero_counters()) != RT_OK) return rc;
        // per-launch timing needs one in-order stream
        const bool timed = (o->flags & RT_TIME_KERNELS) != 0 && n_lanes == 1;
        LaunchMarks marks, marks_b[kMaxBStreams];
        for (int i = -1; i < kMaxBStreams; ++i) {
            LaunchMarks* m = i < 0 ? &marks : &marks_b[i];
            m->pool = &c->tev;
            m->used = &c->t_used;
            m->out = &c->tint;
        }
        // the chain on the caller's stream (tuning chain_on_caller, one lane), or on the lane's own
        // (high-priority) stream after a fork from the caller's; the b streams need no fork: their
        // first work waits for the chain's generation 0 (near_done), which comes after it
        const bool on_caller = c->t(kTuneChainOnCaller) != 0 && n_lanes == 1;
        c->ev0_set = !c->skip_ev0;
        if (c->ev0_set) HIP_TRY(c, hipEventRecord(c->ev0, st));
        if (!on_caller) {
            HIP_TRY(c, hipEventRecord(c->fork, st));
            for (int l = 0; l < n_lanes; ++l) HIP_TRY(c, hipStreamWaitEvent(c->lanes[l].s, c->fork, 0));
        }
        for (uint32_t ci = 0; ci < n_chunks; ++ci) {
            rt_ctx::Lane& L = c->lanes[ci % n_lanes];
            if (ci > 0 && n_lanes > 1) HIP_TRY(c, hipStreamWaitEvent(L.s, c->lanes[(ci - 1) % n_lanes].mark, 0));
            FrameParams f = fp;
            f.row0 = chunk_row0(ci);
            f.rows = chunk_nrows(ci);
            WfBufs b = L.b;
            b.slots = tiles_x * 64 * ((f.rows + 7) / 8);
            WfStreams ws{};
            ws.a = on_caller ? st : L.s;
            ws.nb = split ? n_b : 1;
            for (int i = 0; i < ws.nb; ++i) {
                ws.b[i] = split ? L.sb[i] : ws.a;
                ws.b_done[i] = split ? L.b_done[i] : nullptr;
                ws.mb[i] = timed ? (split ? &marks_b[i] : &marks) : nullptr;
            }
            ws.near_done = L.near_done.data();
            // fused tail (tuning tail_fuse = T): the src-9 tree and light-view grid shadows
            {
                // auto: from generation 4 for chunks of <= 4.5 M pixel slots (one rank's share of a 4- or
                // 8-way C3 frame), from 5 up to 9 M (a 2-way share); with the tail's own fold on one box:
                // 8-way share 0.855 -> 0.751 ms, 4-way 1.140 -> 1.040, 2-way 1.725 -> 1.642 (round 5
                // re-check: 4-way T 5 / 6 1.030 / 1.052 vs 1.039, 2-way T 6 / 7 1.675 / 1.683 vs 1.636-1.642)
                const uint64_t S = static_cast<uint64_t>(tiles_x) * 64u * (chunk_rows / 8);
                int T = static_cast<int>(c->t(kTuneTailFuse));
                // above 9 M slots (the whole C3 frame): from generation max_depth - 1 when that is
                // >= 4 (round 5, depth 8: T = 7 2.898-2.902 vs 2.943-2.945 ms without the tail; 6 /
                // 8 / 9: 2.961 / 2.947-2.960 / 2.970 ms)
                if (T < 0) {
                    const int late = static_cast<int>(o->max_depth) - 1;
                    T = S <= 4500000u ? 4 : S <= 9000000u ? 5 : (late >= 4 ? late : 0);
                }
                const bool ok = T >= 1 && static_cast<uint32_t>(T) <= o->max_depth + 1 && src == 9 && c->all_lights_gridded &&
                                c->t(kTuneGridOcc) != 0;
                ws.tail_fuse = ok ? T : 0;
                ws.tail_width = static_cast<int>(c->t(kTuneTailWidth));
                ws.tail_wgs = static_cast<int>(std::min<uint32_t>(G, static_cast<uint32_t>(c->n_cu)));
            }
            ws.ma = timed ? &marks : nullptr;
            if (split && c->t(kTuneDevJoin)) {
                ws.dj_flags = L.dj;
                ws.dj_next = &L.dj_n;
                ws.dj_err = L.dj_err_dev;
                c->dj_used = true;
            }
            ws.lazy_tally = lazy_tally;
            if (ws.lazy_tally) {
                c->tally.on = true;
                c->tally.zero = !count;         // (a counted render zeroed them above: its test counts are in them)
                c->tally.fp = f;
                c->tally.b = b;
                c->tally.n_lights = c->dsc.n_lights;
                c->tally.gens = static_cast<int>(o->max_depth) + 2;
            }
            ws.cam = cam;
            ws.fold_ev = c->n_bands == 0 ? nullptr : &c->band_ev[ci];
            if (c->sparse_on) {
                ws.sp_s = c->copy_stream;
                ws.sp_cam = c->sp_cam;
                ws.sp_ready = c->sp_ready;
                ws.sp_bits = c->d_sp_bits; ws.sp_cnt = c->d_sp_cnt; ws.sp_off = c->d_sp_off;
                ws.sp_bgr = fp.out_bgr ? c->d_sp_bgr : nullptr;
                ws.sp_rgb = fp.out_rgb ? c->d_sp_rgb : nullptr;
            }
            // every light gridded: the shadow kernel without a tree walk (spheres staged in LDS when
            // they fit in 64 KB); tuning "grid_occ" 0 keeps the general kernel
            ws.grid_occ = (c->all_lights_gridded && c->t(kTuneGridOcc) != 0)
                              ? (static_cast<size_t>(c->dsc.n_spheres) * sizeof(DevSphere) <= 64 * 1024 ? 1 : 2)
                              : 0;
            HIP_TRY(c, launch_wavefront(c->dsc, f, b, src, src_occ, count, ws, L.mark, mark_gen));
        }
        for (int l = 0; l < n_lanes && !on_caller; ++l) {
            HIP_TRY(c, hipEventRecord(c->lanes[l].done, c->lanes[l].s));
            HIP_TRY(c, hipStreamWaitEvent(st, c->lanes[l].done, 0));
        }
        c->wf_used = true;
    } else if (mode == RT_ALGO_PATH) {
        // persistent grid: enough work-items to fill every CU; each owns one
        // recursion stack of max_depth + 1 frames (PathStack)
        const uint64_t npix = static_cast<uint64_t>(o->tile_w) * o->tile_h;
        // work-items per CU = the kernel's occupancy (4 SIMDs x waves per SIMD x 64 lanes)
        const uint32_t T_full = static_cast<uint32_t>(c->n_cu) * 256u * static_cast<uint32_t>(path_waves_per_simd());
        // lanes per pixel: enough work-items to fill the chip, at most one per AA sample
        uint32_t G = 1;
        while (G < 64 && 2 * G <= spp && npix * G < T_full) G *= 2;
        if (const int64_t ge = c->t(kTunePathGroup)) G = static_cast<uint32_t>(ge);   // A/B override
        if (G == 0 || (G & (G - 1)) || G > 64) G = 1;
        fp.path_group = G;
        const uint32_t T = static_cast<uint32_t>(std::min<uint64_t>(T_full, (npix * G + 255) / 256 * 256));
        PathStack ps{};
        ps.T = T;
        ps.levels = o->max_depth + 1;
        const size_t need = PathStack::bytes(T, ps.levels);
        if (need > c->path_bytes) {
            HIP_TRY(c, hipStreamSynchronize(st));
            if (c->d_path) (void)hipFree(c->d_path);
            c->d_path = nullptr;
            c->path_bytes = 0;
            HIP_TRY(c, hipMalloc(&c->d_path, need));
            c->path_bytes = need;
        }
        ps.mem = static_cast<unsigned char*>(c->d_path);
        if (dry) return warm_streams(c, {st});
        if ((rc = zero_counters()) != RT_OK) return rc;
        const bool staged = path_lds_bytes(c->dsc, true) <= 48 * 1024;
        c->ev0_set = true;
        HIP_TRY(c, hipEventRecord(c->ev0, st));
        HIP_TRY(c, launch_path(c->dsc, fp, ps, staged, st));
    } else {
        if (dry) return warm_streams(c, {st});
        if ((rc = zero_counters()) != RT_OK) return rc;
        c->ev0_set = true;
        HIP_TRY(c, hipEventRecord(c->ev0, st));
        HIP_TRY(c, launch_trace_frame(c->dsc, fp, mode, st));
    }
    // the chain schedules (wavefront, megakernel) trace one camera ray tree per
    // pixel and count it spp times: the spp centre-jitter samples are identical
    if (mode != RT_ALGO_PATH) c->last_spp_traced = spp;
    HIP_TRY(c, hipEventRecord(c->render_done, st));
    c->done_stream = st;
    c->render_pending = true;
    c->last_timed = true;
    return RT_OK;
}

int rt_render_device(rt_ctx* c, const rt_render_opts* o, void* d_rgb, void* d_bgr, void* stream) {
    if (!c) return RT_E_INVALID;
    c->skip_ev0 = o && !(o->flags & (RT_TIME_KERNELS | RT_COUNT_WORK));
    const int rc = guarded(c, [&] { return render_device(c, o, d_rgb, d_bgr, stream); });
    c->skip_ev0 = false;
    return rc;
}

int rt_div_a2_check(rt_ctx* c, const double* x, const double* a, uint32_t n, double* fast, double* slow) {
    if (!c || (n && (!x || !a || !fast || !slow))) return RT_E_INVALID;
    if (n == 0) return RT_OK;
    return guarded(c, [&] {
        HIP_TRY(c, hipSetDevice(c->device));
        const size_t bytes = static_cast<size_t>(n) * sizeof(double);
        double* d = nullptr;
        HIP_TRY(c, hipMalloc(&d, 4 * bytes));
        auto body = [&]() -> int {
            HIP_TRY(c, hipMemcpyAsync(d, x, bytes, hipMemcpyHostToDevice, c->stream));
            HIP_TRY(c, hipMemcpyAsync(d + n, a, bytes, hipMemcpyHostToDevice, c->stream));
            HIP_TRY(c, launch_div_a2_probe(d, d + n, n, d + 2 * static_cast<size_t>(n), d + 3 * static_cast<size_t>(n), c->stream));
            HIP_TRY(c, hipMemcpyAsync(fast, d + 2 * static_cast<size_t>(n), bytes, hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(c, hipMemcpyAsync(slow, d + 3 * static_cast<size_t>(n), bytes, hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(c, hipStreamSynchronize(c->stream));
            return RT_OK;
        };
        const int rc = body();
        (void)hipFree(d);
        return rc;
    });
}

int rt_sqrt_check(rt_ctx* c, const double* x, uint32_t n, double* fast, double* slow) {
    if (!c || (n && (!x || !fast || !slow))) return RT_E_INVALID;
    if (n == 0) return RT_OK;
    return guarded(c, [&] {
        HIP_TRY(c, hipSetDevice(c->device));
        const size_t bytes = static_cast<size_t>(n) * sizeof(double);
        double* d = nullptr;
        HIP_TRY(c, hipMalloc(&d, 3 * bytes));
        auto body = [&]() -> int {
            HIP_TRY(c, hipMemcpyAsync(d, x, bytes, hipMemcpyHostToDevice, c->stream));
            HIP_TRY(c, launch_sqrt_probe(d, n, d + n, d + 2 * static_cast<size_t>(n), c->stream));
            HIP_TRY(c, hipMemcpyAsync(fast, d + n, bytes, hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(c, hipMemcpyAsync(slow, d + 2 * static_cast<size_t>(n), bytes, hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(c, hipStreamSynchronize(c->stream));
            return RT_OK;
        };
        const int rc = body();
        (void)hipFree(d);
        return rc;
    });
}

// The tally a one-chunk render left pending, after that render, on the context's stream.
static int flush_tally(rt_ctx* c) {
    if (!c->tally.on) return RT_OK;
    c->tally.on = false;
    HIP_TRY(c, hipStreamWaitEvent(c->stream, c->render_done, 0));
    if (c->tally.zero) HIP_TRY(c, hipMemsetAsync(c->d_counters, 0, kCounterWords * sizeof(unsigned long long), c->stream));
    HIP_TRY(c, launch_tally(c->tally.fp, c->tally.b, c->tally.n_lights, c->tally.gens, c->stream));
    return RT_OK;
}

// A device-side join that gave up (wf_join's 2 s limit) since the last check: reported once (the
// error word is cleared), by the rt_render whose synchronisation follows it or by rt_ctx_stats.
// Only contexts whose renders joined on the device have anything to read (c->dj_used).
static int check_join_error(rt_ctx* c) {
    if (!c->dj_used) return RT_OK;
    for (auto& L : c->lanes) {
        if (!L.dj_err || !__atomic_load_n(L.dj_err, __ATOMIC_ACQUIRE)) continue;
        __atomic_store_n(L.dj_err, 0ull, __ATOMIC_RELEASE);
        return fail(c, RT_E_HIP, "a device-side stream join timed out (tuning dev_join): the render's results are not valid");
    }
    return RT_OK;
}

int rt_ctx_stats(rt_ctx* c, rt_stats* s) {
    if (!c || !s) return RT_E_INVALID;
    HIP_TRY(c, hipSetDevice(c->device));
    if (const int rc = flush_tally(c); rc != RT_OK) return rc;
    unsigned long long h[kCounterWords];
    if (c->last_stream) HIP_TRY(c, hipStreamSynchronize(c->last_stream));
    HIP_TRY(c, hipMemcpyAsync(h, c->d_counters, sizeof h, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    std::memset(s, 0, sizeof *s);
    for (int i = 0; i < kCounterShards; ++i) { s->rays += h[i]; s->shadow_rays += h[kCounterShards + i]; }
    s->rays += h[kTotals] + h[kTotals + 1];
    s->shadow_rays += h[kTotals + 1];
    s->box_tests = h[kTotals + 2] + h[kTotals + 4];
    s->sphere_tests = h[kTotals + 3] + h[kTotals + 5];
    s->shadow_box_tests = h[kTotals + 4];
    s->shadow_sphere_tests = h[kTotals + 5];
    s->pixels = c->last_pixels;
    s->traced_rays = c->last_spp_traced > 1 ? s->rays / c->last_spp_traced : s->rays;
    s->chunks = c->last_chunks;
    if (const int rc = check_join_error(c); rc != RT_OK) return rc;
    if (c->last_timed && c->ev0_set) {
        float ms = 0.f;
        HIP_TRY(c, hipEventSynchronize(c->render_done));
        HIP_TRY(c, hipEventElapsedTime(&ms, c->ev0, c->render_done));
        s->kernel_ms = ms;
    }
    return RT_OK;
}

int rt_ctx_generation_counts(rt_ctx* c, uint32_t* queue, uint32_t* shaded, int n) {
    if (!c || n < 0 || (n && (!queue || !shaded))) return RT_E_INVALID;
    if (!c->wf_used) return fail(c, RT_E_NOSCENE, "no wavefront render yet");
    HIP_TRY(c, hipSetDevice(c->device));
    if (const int rc = flush_tally(c); rc != RT_OK) return rc;
    if (c->last_stream) HIP_TRY(c, hipStreamSynchronize(c->last_stream));
    unsigned long long h[kCntWords];
    HIP_TRY(c, hipMemcpyAsync(h, c->d_counters + kGenTotals, sizeof h, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    for (int k = 0; k < n && k < kCntS; ++k) {
        queue[k] = static_cast<uint32_t>(h[kCntQ + k]);
        shaded[k] = static_cast<uint32_t>(h[kCntS + k]);
    }
    return RT_OK;
}

int rt_ctx_kernel_times(rt_ctx* c, double* ms, uint32_t* launches, int n) {
    if (!c || n < 0 || (n && (!ms || !launches))) return RT_E_INVALID;
    for (int i = 0; i < n; ++i) { ms[i] = 0.0; launches[i] = 0; }
    HIP_TRY(c, hipSetDevice(c->device));
    if (c->t_used > 0) HIP_TRY(c, hipEventSynchronize(c->tev[c->t_used - 1]));
    for (const LaunchInterval& iv : c->tint) {
        float e = 0.f;
        HIP_TRY(c, hipEventElapsedTime(&e, c->tev[iv.start], c->tev[iv.end]));
        if (iv.fam < n) { ms[iv.fam] += e; ++launches[iv.fam]; }
    }
    c->tint.clear();
    c->t_used = 0;
    return RT_OK;
}

// ---- SDMA copy engines (tuning copy_engine) --------------------------------------------
// hipMemcpyAsync moves rt_render's frame to the host at ~29 GB/s on the boxes measured
// (tools/sdma_probe.hip: a blit kernel or the runtime's choice of engine), one SDMA engine
// driven directly at ~53 GB/s.  The engine's queue does not see HIP events, so the host waits
// for the event a copy depends on (hipEventSynchronize) before it queues the copy; each batch
// of copies completes a signal the host waits on.
static hsa_status_t sdma_find_agents(hsa_agent_t a, void* data) {
    auto* c = static_cast<rt_ctx*>(data);
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
    if (t == HSA_DEVICE_TYPE_CPU && c->hsa_cpu.handle == 0) c->hsa_cpu = a;
    if (t == HSA_DEVICE_TYPE_GPU && c->hsa_gpu.handle == 0) {
        // the HIP device's agent: same PCI domain, bus and device
        uint32_t bdf = 0, dom = 0;
        int bus = -1, dev = -1, hdom = -1;
        (void)hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf);
        (void)hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &dom);
        if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, c->device) == hipSuccess &&
            hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, c->device) == hipSuccess &&
            hipDeviceGetAttribute(&hdom, hipDeviceAttributePciDomainID, c->device) == hipSuccess &&
            static_cast<int>((bdf >> 8) & 0xFF) == bus && static_cast<int>((bdf >> 3) & 0x1F) == dev &&
            static_cast<int>(dom) == hdom)
            c->hsa_gpu = a;
        (void)hipGetLastError();
    }
    return HSA_STATUS_SUCCESS;
}

// Set up once per context; false if the device has no usable engine (the HIP path is used).
static bool sdma_setup(rt_ctx* c) {
    if (c->sdma_state) return c->sdma_state == 1;
    c->sdma_state = -1;
    if (hsa_init() != HSA_STATUS_SUCCESS) return false;
    bool ok = hsa_iterate_agents(sdma_find_agents, c) == HSA_STATUS_SUCCESS && c->hsa_gpu.handle && c->hsa_cpu.handle &&
              hsa_amd_memory_copy_engine_status(c->hsa_cpu, c->hsa_gpu, &c->sdma_avail) == HSA_STATUS_SUCCESS &&
              c->sdma_avail != 0;
    if (ok && hsa_amd_memory_get_preferred_copy_engine(c->hsa_cpu, c->hsa_gpu, &c->sdma_pref) != HSA_STATUS_SUCCESS)
        c->sdma_pref = 0;
    for (int i = 0; ok && i < rt_ctx::kSdmaSignals; ++i) ok = hsa_signal_create(0, 0, nullptr, &c->sdma_sig[i]) == HSA_STATUS_SUCCESS;
    if (!ok) {
        for (hsa_signal_t& sg : c->sdma_sig)
            if (sg.handle) { (void)hsa_signal_destroy(sg); sg.handle = 0; }
        (void)hsa_shut_down();
        return false;
    }
    c->sdma_state = 1;
    return true;
}

// The engines rt_render's copies use now, as a mask taken in turn (0: hipMemcpyAsync).  -1: the
// device's engines 0-3 (tools/sdma_probe: ~53 GB/s each on MI355X, the PCIe link's rate; engines
// 4-15 move 7-12.5 GB/s); several in turn hide each copy's fixed cost behind the others' transfers
// (a rank's 64 row bands of 192 KB: 38 GB/s on four engines, 14 GB/s on one).
static uint32_t sdma_engine(rt_ctx* c) {
    int64_t e = c->t(kTuneCopyEngine);
    if (e == -2) e = c->copy_banded ? -1 : 0;
    if (e == 0 || !sdma_setup(c)) return 0;
    if (e > 0) return (1u << (e - 1)) & c->sdma_avail;
    if (c->sdma_avail & 0xFu) return c->sdma_avail & 0xFu;
    const uint32_t m = (c->sdma_pref & c->sdma_avail) ? (c->sdma_pref & c->sdma_avail) : c->sdma_avail;
    return m & (~m + 1u);
}

// Wait until signal `si` is 0 (every copy counted on it done); a copy that has not completed
// after 30 s is an error, not a hang.
static int sdma_wait(rt_ctx* c, int si) {
    static const uint64_t hint = [] {
        uint64_t f = 0;
        return hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &f) == HSA_STATUS_SUCCESS && f ? f / 1000 : 1000000;
    }();
    const auto t0 = std::chrono::steady_clock::now();
    while (hsa_signal_wait_scacquire(c->sdma_sig[si], HSA_SIGNAL_CONDITION_EQ, 0, hint, HSA_WAIT_STATE_ACTIVE) != 0)
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30))
            return fail(c, RT_E_HIP, "an SDMA copy did not complete");
    return RT_OK;
}

// Device -> pinned host copy on the next engine of `engines` (in turn), counted on signal `si` (one
// more pending copy); the caller waits with sdma_wait.  Copies on different engines complete in
// any order: a wait covers exactly the copies counted on its signal.
static int sdma_copy(rt_ctx* c, uint32_t engines, int si, void* dst, const void* src, size_t bytes) {
    if (!bytes) return RT_OK;
    uint32_t engine = 0;
    for (int k = 0; k < 32 && !engine; ++k) {
        const uint32_t bit = 1u << (c->sdma_turn++ & 31u);
        if (engines & bit) engine = bit;
    }
    hsa_signal_t sg = c->sdma_sig[si];
    hsa_signal_add_screlease(sg, 1);
    const hsa_status_t st = hsa_amd_memory_async_copy_on_engine(dst, c->hsa_cpu, src, c->hsa_gpu, bytes, 0, nullptr, sg,
                                                                static_cast<hsa_amd_sdma_engine_id_t>(engine), true);
    if (st != HSA_STATUS_SUCCESS) {
        hsa_signal_subtract_screlease(sg, 1);
        (void)sdma_wait(c, si);              // the copies queued before it still complete
        return fail(c, RT_E_HIP, "hsa_amd_memory_async_copy_on_engine failed (" + std::to_string(st) + ")");
    }
    return RT_OK;
}

// Wait for an event by polling it: a blocking wait's wake-up costs tens of microseconds, which a
// frame of a few hundred microseconds notices at every step of its copies.
static hipError_t spin_wait(hipEvent_t ev) {
    for (;;) {
        const hipError_t e = hipEventQuery(ev);
        if (e != hipErrorNotReady) return e;
        std::this_thread::yield();
    }
}

// Where rt_render puts a device row (RT_OUT_FRAME_ROWS or not): local row j of the tile, dev_pitch
// bytes apart on the device, row_bytes of it copied, lands at host byte offset host_row(j) *
// host_pitch + host_x.  A plain tile: host_row(j) = j, the host rows laid out as the device's; a
// frame: the tile's frame row (rt_render_opts: y0 + ((j/band)*band_stride + band_phase)*band + j%band).
struct OutMap {
    size_t dev_pitch = 0, row_bytes = 0, host_pitch = 0, host_x = 0;
    bool frame = false;
    uint32_t y0 = 0, band = 1, stride = 1, phase = 0;
    size_t host_row(uint32_t j) const {
        return frame ? y0 + (static_cast<size_t>(j / band) * stride + phase) * band + j % band : j;
    }
    size_t host_off(uint32_t j) const { return host_row(j) * host_pitch + host_x; }
    // consecutive rows are one contiguous byte range on both sides
    bool contiguous() const { return dev_pitch == host_pitch && row_bytes == dev_pitch && host_x == 0; }
    // local rows j and j + 1 sit in consecutive host rows
    bool next_row(uint32_t j) const { return host_row(j + 1) == host_row(j) + 1; }
};

// Device -> caller-owned host memory, row band by row band: the copy stream
// waits for each band's fold (c->band_ev, recorded by the render when
// c->want_bands was set; otherwise for the whole render), so the PCIe transfer
// of the first bands overlaps the fold of the later ones.  A page-locked
// destination gets the DMA directly (one copy per run of rows that are
// consecutive on the host, 2D when the rows are not back to back); pageable
// memory goes through kRing pinned slices of whole rows, the copy engine
// filling slices ahead while the host pool empties them in order into their
// host rows.  wait = false (sparse copies): no wait on the bands, the copy
// stream's order alone (its segment kernels follow the camera pass).
static int copy_to_host(rt_ctx* c, void* dst, const void* src, const OutMap& m, uint32_t rows, hipEvent_t after = nullptr,
                        bool sync = true) {
    if (!rows || !m.row_bytes) return RT_OK;
    int rc = ensure_copy_stream(c);
    if (rc != RT_OK) return rc;
    if (!c->cp_done) HIP_TRY(c, hipEventCreateWithFlags(&c->cp_done, hipEventDisableTiming));
    const uint32_t engine = sdma_engine(c);          // 0: hipMemcpyAsync on the copy stream
    const auto* s8 = static_cast<const uint8_t*>(src);
    auto* d8 = static_cast<uint8_t*>(dst);
    hipPointerAttribute_t attr{};
    const bool pinned = hipPointerGetAttributes(&attr, dst) == hipSuccess && attr.type == hipMemoryTypeHost;
    (void)hipGetLastError();                       // a pageable pointer is not an error
    const bool contig = m.contiguous();
    // pieces: rows [j0, j0 + n) of one chunk band, consecutive on the host (pinned), at most one
    // staging slice of rows (pageable)
    const size_t slice = std::max(kSlice, m.dev_pitch);
    const uint32_t slice_rows = static_cast<uint32_t>(std::max<size_t>(1, slice / m.dev_pitch));
    struct Piece { uint32_t j0, n; int band; };
    std::vector<Piece> pieces;
    const int nb = c->n_bands > 0 ? c->n_bands : 1;
    for (int bi = 0; bi < nb; ++bi) {
        const uint32_t a = c->n_bands > 0 ? c->band_row0[bi] : 0;
        const uint32_t e = c->n_bands > 0 ? std::min(rows, c->band_row0[bi] + c->band_nrows[bi]) : rows;
        for (uint32_t j = a; j < e;) {
            uint32_t n = 1;
            if (pinned) {
                while (j + n < e && m.next_row(j + n - 1) && (contig || n < 65535)) ++n;
            } else {
                n = std::min(slice_rows, e - j);
            }
            pieces.push_back(Piece{j, n, bi});
            j += n;
        }
    }
    // a piece is copied once its chunk band is final (band_ev; the whole render: render_done),
    // or after `after`: the copy stream waits for the event, the host for an engine's copies
    auto band_event = [&](int bi) { return after ? after : c->n_bands > 0 ? c->band_ev[bi] : c->render_done; };
    auto wait_band = [&](int bi) -> hipError_t {
        return engine ? hipEventSynchronize(band_event(bi)) : hipStreamWaitEvent(c->copy_stream, band_event(bi), 0);
    };
    // page-locked destination: every piece straight into the caller's rows, one copy per piece (the
    // rows of a partial-width tile: one per row), on the engines or the copy stream.  (Not
    // hipMemcpy2DAsync: a 2D copy of rows whose length is not a multiple of 4 was seen to land
    // after the stream's later event, tools/copy_stress.py.)
    if (pinned) {
        constexpr int si = rt_ctx::kSdmaSignals - 1;
        int last = -1;
        for (const Piece& pc : pieces) {
            if (pc.band != last) { HIP_TRY(c, wait_band(pc.band)); last = pc.band; }
            for (uint32_t j = pc.j0; j < pc.j0 + pc.n; j += contig ? pc.n : 1) {
                void* to = d8 + m.host_off(j);
                const void* from = s8 + j * m.dev_pitch;
                const size_t len = contig ? pc.n * m.dev_pitch : m.row_bytes;
                if (engine) {
                    if ((rc = sdma_copy(c, engine, si, to, from, len)) != RT_OK) return rc;
                } else {
                    HIP_TRY(c, hipMemcpyAsync(to, from, len, hipMemcpyDeviceToHost, c->copy_stream));
                }
            }
        }
        if (!sync) return RT_OK;
        if (engine) return sdma_wait(c, si);
        HIP_TRY(c, hipEventRecord(c->cp_done, c->copy_stream));
        HIP_TRY(c, spin_wait(c->cp_done));
        return RT_OK;
    }
    if (slice > c->pin_cap) {                      // rows wider than a slice: larger slices
        for (int i = 0; i < kRing; ++i) {
            if (c->pin[i]) (void)hipHostFree(c->pin[i]);
            c->pin[i] = nullptr;
        }
        c->pin_cap = slice;
    }
    for (int i = 0; i < kRing; ++i) {
        if (!c->pin[i]) HIP_TRY(c, hipHostMalloc(&c->pin[i], c->pin_cap, hipHostMallocDefault));
        if (!c->pin_ev[i]) HIP_TRY(c, hipEventCreateWithFlags(&c->pin_ev[i], hipEventDisableTiming));
    }
    const size_t n = pieces.size();
    size_t issued = 0, drained = 0;
    int last = -1;
    while (drained < n) {
        while (issued < n && issued - drained < static_cast<size_t>(kRing)) {   // slot issued % kRing is free
            const Piece& pc = pieces[issued];
            if (pc.band != last) { HIP_TRY(c, wait_band(pc.band)); last = pc.band; }
            const int slot = static_cast<int>(issued % kRing);
            if (engine) {
                if ((rc = sdma_copy(c, engine, slot, c->pin[slot], s8 + pc.j0 * m.dev_pitch, pc.n * m.dev_pitch)) != RT_OK)
                    return rc;
            } else {
                HIP_TRY(c, hipMemcpyAsync(c->pin[slot], s8 + pc.j0 * m.dev_pitch, pc.n * m.dev_pitch, hipMemcpyDeviceToHost,
                                          c->copy_stream));
                HIP_TRY(c, hipEventRecord(c->pin_ev[slot], c->copy_stream));
            }
            ++issued;
        }
        const int slot = static_cast<int>(drained % kRing);
        if (engine) {
            if ((rc = sdma_wait(c, slot)) != RT_OK) return rc;
        } else {
            HIP_TRY(c, spin_wait(c->pin_ev[slot]));
        }
        const Piece& pc = pieces[drained];
        const auto* from = static_cast<const uint8_t*>(c->pin[slot]);
        if (!m.frame && contig) {
            c->pool.copy(d8 + m.host_off(pc.j0), from, pc.n * m.dev_pitch);
        } else {                                   // row by row into the host rows, shared by the pool
            const size_t parts = std::min<size_t>(HostCopyPool::kParts, pc.n);
            c->pool.run(parts, [&](size_t q) {
                const uint32_t a = pc.j0 + static_cast<uint32_t>(pc.n * q / parts), e = pc.j0 + static_cast<uint32_t>(pc.n * (q + 1) / parts);
                for (uint32_t j = a; j < e; ++j) std::memcpy(d8 + m.host_off(j), from + (j - pc.j0) * m.dev_pitch, m.row_bytes);
            });
        }
        ++drained;
    }
    return RT_OK;
}

// Pinned host buffer of at least `bytes` (grown on demand).
static int ensure_pinned(rt_ctx* c, void*& p, size_t& cap, size_t bytes) {
    if (bytes <= cap) return RT_OK;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    HIP_TRY(c, hipHostMalloc(&p, bytes, hipHostMallocDefault));
    cap = bytes;
    return RT_OK;
}

// rt_render's copies after a sparse render: the row offsets and segment bits,
// then the whole frame as the camera pass left it (every pixel without a chain is final; the
// generations run meanwhile), then, once the render is done, the packed chain segments in row
// ranges, each scattered into the host rows by the host pool as soon as it has landed.
static int copy_sparse(rt_ctx* c, const rt_render_opts* o, float* out_rgb, uint8_t* out_bgr, const OutMap& mr,
                       const OutMap& mb) {
    const uint32_t rows = o->tile_h, tw = o->tile_w;
    const uint32_t nseg = (tw + kSegPx - 1) / kSegPx, words = (nseg + 31) / 32;
    const size_t s_off = (rows + 1ull) * 4, s_bits = static_cast<size_t>(rows) * words * 4;
    using Clock = std::chrono::steady_clock;
    const auto t0 = Clock::now();
    auto us = [&] { return std::chrono::duration<double, std::micro>(Clock::now() - t0).count(); };
    int rc = ensure_pinned(c, c->h_sp_meta, c->h_sp_meta_cap, s_off + s_bits);
    if (rc != RT_OK) return rc;
    auto* h_off = static_cast<uint32_t*>(c->h_sp_meta);
    auto* h_bits = h_off + (rows + 1);
    HIP_TRY(c, hipMemcpyAsync(h_off, c->d_sp_off, s_off, hipMemcpyDeviceToHost, c->copy_stream));
    HIP_TRY(c, hipMemcpyAsync(h_bits, c->d_sp_bits, s_bits, hipMemcpyDeviceToHost, c->copy_stream));
    if (!c->cp_done) HIP_TRY(c, hipEventCreateWithFlags(&c->cp_done, hipEventDisableTiming));
    HIP_TRY(c, hipEventRecord(c->cp_done, c->copy_stream));          // the offsets and bits have landed
    // the frame as the camera pass left it (sp_ready: after the segment kernels, which follow the camera pass):
    // into a page-locked frame the copies are only queued here (the packed ranges queue behind them and
    // the host waits for those), into pageable memory the staging slices are drained as they land
    const uint32_t engine = sdma_engine(c);
    if (out_bgr && (rc = copy_to_host(c, out_bgr, c->d_bgr, mb, rows, c->sp_ready, false)) != RT_OK) return rc;
    if (out_rgb && (rc = copy_to_host(c, out_rgb, c->d_rgb, mr, rows, c->sp_ready, false)) != RT_OK) return rc;
    const double t_queued = us();
    HIP_TRY(c, spin_wait(c->cp_done));
    const double t_frame = us();
    const uint64_t total = h_off[rows];
    const size_t seg_b = 3 * kSegPx, seg_r = 3 * kSegPx * sizeof(float);
    const size_t pk_b = out_bgr ? total * seg_b : 0, pk_r = out_rgb ? total * seg_r : 0;
    if ((rc = ensure_pinned(c, c->h_sp_pk, c->h_sp_pk_cap, std::max<size_t>(1, pk_b + pk_r))) != RT_OK) return rc;
    auto* hb = static_cast<uint8_t*>(c->h_sp_pk);
    auto* hr = reinterpret_cast<float*>(hb + pk_b);
    // the packed segments once the render is done: on the copy stream after its end event, or on the
    // engine once the host has seen it, in row ranges, each with its own event / signal
    const hipEvent_t done = c->n_bands > 0 ? c->band_ev[0] : c->render_done;
    if (engine) HIP_TRY(c, spin_wait(done));
    else HIP_TRY(c, hipStreamWaitEvent(c->copy_stream, done, 0));
    const double t_done = us();
    // ranges of at least ~2 MB (each copy has a fixed cost of its own), at most kSpRanges
    const int nr = static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>({static_cast<uint64_t>(rt_ctx::kSpRanges), rows,
                                                                             (pk_b + pk_r + (2u << 20) - 1) / (2u << 20)})));
    auto r_at = [&](int j) { return static_cast<uint32_t>(static_cast<uint64_t>(rows) * j / nr); };
    for (int j = 0; j < nr; ++j) {
        const uint64_t a = h_off[r_at(j)], e = h_off[r_at(j + 1)];
        if (engine) {
            if (e > a && out_bgr && (rc = sdma_copy(c, engine, kRing + j, hb + a * seg_b, c->d_sp_bgr + a * seg_b, (e - a) * seg_b)) != RT_OK)
                return rc;
            if (e > a && out_rgb &&
                (rc = sdma_copy(c, engine, kRing + j, hr + a * 3 * kSegPx, c->d_sp_rgb + a * 3 * kSegPx, (e - a) * seg_r)) != RT_OK)
                return rc;
            continue;
        }
        if (!c->sp_ev[j]) HIP_TRY(c, hipEventCreateWithFlags(&c->sp_ev[j], hipEventDisableTiming));
        if (e > a && out_bgr)
            HIP_TRY(c, hipMemcpyAsync(hb + a * seg_b, c->d_sp_bgr + a * seg_b, (e - a) * seg_b, hipMemcpyDeviceToHost, c->copy_stream));
        if (e > a && out_rgb)
            HIP_TRY(c, hipMemcpyAsync(hr + a * 3 * kSegPx, c->d_sp_rgb + a * 3 * kSegPx, (e - a) * seg_r, hipMemcpyDeviceToHost,
                                      c->copy_stream));
        HIP_TRY(c, hipEventRecord(c->sp_ev[j], c->copy_stream));
    }
    const size_t pad = mb.row_bytes - 3ull * tw;           // BMP row padding of the tile's rows (device pitch)
    auto* rgb8 = reinterpret_cast<uint8_t*>(out_rgb);
    auto scatter_rows = [&](uint32_t r0, uint32_t r1) {
        for (uint32_t r = r0; r < r1; ++r) {
            const uint32_t* bits = h_bits + static_cast<size_t>(r) * words;
            uint64_t i = h_off[r];
            for (uint32_t w = 0; w < words; ++w)
                for (uint32_t m = bits[w]; m; m &= m - 1, ++i) {
                    const uint32_t x0 = (w * 32 + static_cast<uint32_t>(__builtin_ctz(m))) * kSegPx;
                    const uint32_t n = std::min(kSegPx, tw - x0);
                    if (out_bgr) {
                        uint8_t* d = out_bgr + mb.host_off(r) + 3ull * x0;
                        std::memcpy(d, hb + i * seg_b, 3ull * n);
                        if (x0 + n == tw && pad) std::memset(d + 3ull * n, 0, pad);   // BMP row padding
                    }
                    if (out_rgb) std::memcpy(rgb8 + mr.host_off(r) + 12ull * x0, hr + i * 3 * kSegPx, 12ull * n);
                }
        }
    };
    // each range scattered by the pool as soon as it has landed (the later ones still in flight)
    double t_first = 0.0;
    // (engine: the frame's copies were queued on the same engine before the ranges; its signal first)
    if (engine && (rc = sdma_wait(c, rt_ctx::kSdmaSignals - 1)) != RT_OK) return rc;
    for (int j = 0; j < nr; ++j) {
        if (engine) {
            if ((rc = sdma_wait(c, kRing + j)) != RT_OK) return rc;
        } else {
            HIP_TRY(c, spin_wait(c->sp_ev[j]));
        }
        if (j == 0) t_first = us();
        const uint32_t ra = r_at(j), rb = r_at(j + 1);
        const size_t parts = std::min<size_t>(HostCopyPool::kParts, rb - ra);
        c->pool.run(parts, [&](size_t q) {
            scatter_rows(ra + static_cast<uint32_t>((rb - ra) * q / parts), ra + static_cast<uint32_t>((rb - ra) * (q + 1) / parts));
        });
    }
    if (c->t(kTuneVerbose))
        std::fprintf(stderr, "rtamd: sparse copy: %llu of %llu segments; frame copies queued at %.0f us, offsets in at %.0f, "
                     "render done seen at %.0f (engine only), first packed range in at %.0f, done at %.0f\n",
                     static_cast<unsigned long long>(total), static_cast<unsigned long long>(nseg) * rows, t_queued, t_frame,
                     engine ? t_done : 0.0, t_first, us());
    return RT_OK;
}

// rt_render's layout on both sides (check_opts has validated o): the device frame of the tile
// (f32 rows of 12 tile_w bytes, BGR rows of *dev_bgr_pitch bytes) and where each row goes on the host.
static int host_layout(rt_ctx* c, const rt_render_opts* o, uint32_t pitch, OutMap& mr, OutMap& mb, uint32_t* dev_bgr_pitch) {
    const bool frame = (o->flags & RT_OUT_FRAME_ROWS) != 0;
    mr = OutMap{};
    mr.dev_pitch = mr.row_bytes = static_cast<size_t>(o->tile_w) * 12;
    mr.host_pitch = mr.dev_pitch;
    if (frame) {
        const uint32_t hp = o->bgr_pitch ? o->bgr_pitch : 3 * o->width;
        if (hp < 3ull * o->width) return fail(c, RT_E_INVALID, "RT_OUT_FRAME_ROWS: bgr_pitch < 3*width");
        mr.frame = true;
        mr.y0 = o->y0; mr.band = o->band ? o->band : 1; mr.stride = o->band_stride ? o->band_stride : 1; mr.phase = o->band_phase;
        mr.host_pitch = static_cast<size_t>(o->width) * 12;
        mr.host_x = static_cast<size_t>(o->x0) * 12;
        mb = mr;
        // the tile's BGR rows carry the frame's row padding when the tile ends at the frame's right edge
        const uint32_t pad = o->x0 + o->tile_w == o->width ? hp - 3 * o->width : 0;
        mb.dev_pitch = mb.row_bytes = 3ull * o->tile_w + pad;
        mb.host_pitch = hp;
        mb.host_x = 3ull * o->x0;
        *dev_bgr_pitch = 3 * o->tile_w + pad;
    } else {
        mb = OutMap{};
        mb.dev_pitch = mb.row_bytes = mb.host_pitch = pitch;
        *dev_bgr_pitch = pitch;
    }
    return RT_OK;
}

// rt_render's device frame for the tile: grown on demand (an earlier render may still write it).
static int ensure_host_frame(rt_ctx* c, size_t rgb_bytes, size_t bgr_bytes) {
    if (c->render_pending && (rgb_bytes > c->rgb_cap || bgr_bytes > c->bgr_cap))
        HIP_TRY(c, hipEventSynchronize(c->render_done));
    if (rgb_bytes > c->rgb_cap) {
        if (c->d_rgb) (void)hipFree(c->d_rgb);
        c->d_rgb = nullptr; c->rgb_cap = 0;
        HIP_TRY(c, hipMalloc(&c->d_rgb, rgb_bytes));
        c->rgb_cap = rgb_bytes;
    }
    if (bgr_bytes > c->bgr_cap) {
        if (c->d_bgr) (void)hipFree(c->d_bgr);
        c->d_bgr = nullptr; c->bgr_cap = 0;
        HIP_TRY(c, hipMalloc(&c->d_bgr, bgr_bytes));
        c->bgr_cap = bgr_bytes;
    }
    return RT_OK;
}

static int render_host(rt_ctx* c, const rt_render_opts* o, float* out_rgb, uint8_t* out_bgr, rt_stats* stats) {
    uint32_t spp, band, stride, pitch;
    int rc = check_opts(c, o, spp, band, stride, pitch);
    if (rc != RT_OK) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    OutMap mr, mb;
    uint32_t dev_pitch = pitch;
    if ((rc = host_layout(c, o, pitch, mr, mb, &dev_pitch)) != RT_OK) return rc;
    c->copy_banded = stride > 1;
    rt_render_opts oo = *o;
    oo.flags = (o->flags & ~(RT_OUT_RGB_F32 | RT_OUT_BGR_U8 | RT_OUT_FRAME_ROWS)) | (out_rgb ? RT_OUT_RGB_F32 : 0) |
               (out_bgr ? RT_OUT_BGR_U8 : 0);
    oo.bgr_pitch = dev_pitch;
    // an earlier rt_render's copies (copy stream) are done with d_rgb / d_bgr: copy_to_host returns
    // only once its last piece has been drained or synchronised
    if ((rc = ensure_host_frame(c, out_rgb ? mr.dev_pitch * o->tile_h : 0, out_bgr ? mb.dev_pitch * o->tile_h : 0)) != RT_OK)
        return rc;
    c->want_bands = true;
    c->want_sparse = c->t(kTuneSparseOut) != 0;
    rc = render_device(c, &oo, c->d_rgb, c->d_bgr, nullptr);
    c->want_bands = false;
    c->want_sparse = false;
    if (rc != RT_OK) return rc;
    if (c->sparse_on) {
        if ((rc = copy_sparse(c, o, out_rgb, out_bgr, mr, mb)) != RT_OK) return rc;
    } else {
        if (out_bgr && (rc = copy_to_host(c, out_bgr, c->d_bgr, mb, o->tile_h)) != RT_OK) return rc;
        if (out_rgb && (rc = copy_to_host(c, out_rgb, c->d_rgb, mr, o->tile_h)) != RT_OK) return rc;
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (stats) return rt_ctx_stats(c, stats);
    return check_join_error(c);
}

int rt_render(rt_ctx* c, const rt_render_opts* o, float* out_rgb, uint8_t* out_bgr, rt_stats* stats) {
    if (!c || !o) return RT_E_INVALID;
    return guarded(c, [&] { return render_host(c, o, out_rgb, out_bgr, stats); });
}

// rt_ctx_reserve: render_device's allocations and streams without its launches (dry), plus, for
// rt_render (host), the device frame, the staging slices and the sparse copies' pinned buffers.
static int reserve(rt_ctx* c, const rt_render_opts* o, int host, void* stream) {
    if (!c->has_scene) return fail(c, RT_E_NOSCENE, "no scene uploaded");
    uint32_t spp, band, stride, pitch;
    int rc = check_opts(c, o, spp, band, stride, pitch);
    if (rc != RT_OK) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    rt_render_opts oo = *o;
    if (!host) {
        if (o->flags & RT_OUT_FRAME_ROWS) return fail(c, RT_E_INVALID, "RT_OUT_FRAME_ROWS is for rt_render's host buffers");
        return render_device(c, &oo, nullptr, nullptr, stream, true);
    }
    OutMap mr, mb;
    uint32_t dev_pitch = pitch;
    if ((rc = host_layout(c, o, pitch, mr, mb, &dev_pitch)) != RT_OK) return rc;
    c->copy_banded = stride > 1;
    oo.flags &= ~RT_OUT_FRAME_ROWS;
    oo.bgr_pitch = dev_pitch;
    const bool rgb = (o->flags & RT_OUT_RGB_F32) != 0, bgr = (o->flags & RT_OUT_BGR_U8) != 0;
    if ((rc = ensure_host_frame(c, rgb ? mr.dev_pitch * o->tile_h : 0, bgr ? mb.dev_pitch * o->tile_h : 0)) != RT_OK) return rc;
    c->want_bands = true;
    c->want_sparse = c->t(kTuneSparseOut) != 0;
    rc = render_device(c, &oo, c->d_rgb, c->d_bgr, nullptr, true);
    c->want_bands = false;
    c->want_sparse = false;
    if (rc != RT_OK) return rc;
    for (int i = 0; i < kRing; ++i) {               // the staging slices of pageable destinations
        if (!c->pin[i]) HIP_TRY(c, hipHostMalloc(&c->pin[i], c->pin_cap, hipHostMallocDefault));
        if (!c->pin_ev[i]) HIP_TRY(c, hipEventCreateWithFlags(&c->pin_ev[i], hipEventDisableTiming));
    }
    if (c->sparse_on) {
        const uint64_t nseg = (o->tile_w + kSegPx - 1) / kSegPx, words = (nseg + 31) / 32;
        if ((rc = ensure_pinned(c, c->h_sp_meta, c->h_sp_meta_cap, (o->tile_h + 1ull) * 4 + o->tile_h * words * 4)) != RT_OK)
            return rc;
        // the packed segments' pinned buffer at its worst case (every segment flagged), up to 1 GB;
        // a render that needs more grows it
        const uint64_t worst = nseg * o->tile_h * 3 * kSegPx * ((bgr ? 1 : 0) + (rgb ? 4 : 0));
        if ((rc = ensure_pinned(c, c->h_sp_pk, c->h_sp_pk_cap, std::max<uint64_t>(1, std::min<uint64_t>(worst, 1ull << 30)))) != RT_OK)
            return rc;
        for (int j = 0; j < rt_ctx::kSpRanges; ++j)
            if (!c->sp_ev[j]) HIP_TRY(c, hipEventCreateWithFlags(&c->sp_ev[j], hipEventDisableTiming));
    }
    // the copy engine's queue is set up at its first copy (tens of ms): one small copy now
    if (const uint32_t engine = sdma_engine(c)) {
        constexpr int si = rt_ctx::kSdmaSignals - 1;
        if ((rc = sdma_copy(c, engine, si, c->pin[0], c->d_counters, 4096)) != RT_OK || (rc = sdma_wait(c, si)) != RT_OK)
            return rc;
    }
    return RT_OK;
}

int rt_ctx_reserve(rt_ctx* c, const rt_render_opts* o, int host, void* stream) {
    if (!c || !o) return RT_E_INVALID;
    return guarded(c, [&] { return reserve(c, o, host, stream); });
}

int rt_ctx_set_tuning(rt_ctx* c, const char* key, int64_t value) {
    if (!c || !key) return RT_E_INVALID;
    for (int i = 0; i < kTuneCount; ++i) {
        if (std::strcmp(key, kTune[i].name) != 0) continue;
        if (value < kTune[i].lo || value > kTune[i].hi)
            return fail(c, RT_E_INVALID, std::string("tuning ") + key + " out of range");
        // cu_mask and prio shape the lanes' streams, which are created once: rebuild
        // the lanes (after their work is done) so the next render uses the new value
        if ((i == kTuneCuMask || i == kTunePrio || i == kTuneAQueue) && value != c->tune[i] && !c->lanes.empty()) {
            if (hipSetDevice(c->device) != hipSuccess) return fail(c, RT_E_HIP, "hipSetDevice failed");
            if (c->render_pending) (void)hipEventSynchronize(c->render_done);
            drop_lanes(c);
        }
        c->tune[i] = value;
        return RT_OK;
    }
    return fail(c, RT_E_INVALID, std::string("unknown tuning key ") + key);
}

int rt_ctx_get_tuning(const rt_ctx* c, const char* key, int64_t* value) {
    if (!c || !key || !value) return RT_E_INVALID;
    for (int i = 0; i < kTuneCount; ++i)
        if (std::strcmp(key, kTune[i].name) == 0) { *value = c->tune[i]; return RT_OK; }
    return RT_E_INVALID;
}

const char* rt_tuning_key(int index) { return index >= 0 && index < kTuneCount ? kTune[index].name : nullptr; }

}  // extern "C"
