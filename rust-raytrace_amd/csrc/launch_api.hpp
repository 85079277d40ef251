// Host-side launchers of the kernels in trace_kernel.hip (called by rt_device.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "device_layout.hpp"

namespace rtamd {

// Kernel families of the wavefront schedule (rt_ctx_kernel_times indices).
enum KernelFamily : int8_t {
    kKfNearest = 0, kKfOcclusion = 1, kKfShade = 2, kKfFold = 3, kKfTally = 4, kKfCamera = 5, kKfCompose = 6, kKfTail = 7, kKfCount = 8
};

// Per-launch timing (RT_TIME_KERNELS): begin() records a start event before a
// launch (after any cross-stream wait), mark() an end event after it, noting
// (start, end, family): the elapsed time between the two is that launch's
// duration (one LaunchMarks per stream).  Events
// come from a pool owned by the context; intervals accumulate over renders
// until harvested (rt_ctx_kernel_times).
struct LaunchInterval {
    int start, end;
    KernelFamily fam;
};

struct LaunchMarks {
    std::vector<hipEvent_t>* pool = nullptr;
    int* used = nullptr;                   // events of the pool in use
    std::vector<LaunchInterval>* out = nullptr;
    int prev = -1;
    static constexpr int kMaxEvents = 1 << 16;

    hipError_t record(hipStream_t s, int& idx) {
        idx = -1;
        if (*used >= kMaxEvents) return hipSuccess;    // not harvested: stop recording
        if (*used == static_cast<int>(pool->size())) {
            hipEvent_t e;
            const hipError_t err = hipEventCreate(&e);
            if (err != hipSuccess) return err;
            pool->push_back(e);
        }
        idx = (*used)++;
        return hipEventRecord((*pool)[idx], s);
    }
    hipError_t begin(hipStream_t s) { return record(s, prev); }
    hipError_t mark(hipStream_t s, KernelFamily f) {
        int idx;
        const hipError_t e = record(s, idx);
        if (e == hipSuccess && idx >= 0 && prev >= 0) out->push_back(LaunchInterval{prev, idx, f});
        prev = idx;
        return e;
    }
};

hipError_t launch_trace_frame(const DevScene& sc, const FrameParams& fp, int mode, hipStream_t stream);
// The streams of one wavefront lane: a runs the nearest-hit chain and the
// fold; the shadow + shading kernels of generation k run on b[k % nb] (b[i] ==
// a: one in-order stream).  near_done: kMaxGenerations events; b_done: one
// per b stream; marks may be null.  Sphere sources and the supported
// (nearest, shadow) pairs: trace_kernel.hip kSrc* and launch_wavefront.
constexpr int kMaxBStreams = 4;
struct WfStreams {
    hipStream_t a;
    hipStream_t b[kMaxBStreams];
    int nb;
    hipEvent_t* near_done;
    hipEvent_t b_done[kMaxBStreams];
    LaunchMarks* ma;
    LaunchMarks* mb[kMaxBStreams];
    int cam;            // generation 0: 0 per-ray traversal of the nearest-hit source, 3 / 4 the camera's view
                        // grid with the spheres in LDS / through L2
    int grid_occ;       // every light has a light-view grid: shadow kernel without a tree walk,
                        // spheres from LDS (1) or HBM/L2 (2); 0: the general shadow kernel
    hipEvent_t* fold_ev;// recorded once the chunk's pixels are final (null: no event)
    int tail_fuse;        // > 0: the chains running at generation tail_fuse - 1 finish in one wf_tail
    int tail_wgs;         //   launch on stream a (that many workgroups, all resident: one per CU;
    int tail_width;       //   chains per wave, 0 auto), which folds them; the others fold on b[0]
    // sparse host copies (b.mark set): after generation 0 (sp_cam), stream sp_s runs the segment
    // kernels into sp_bits / sp_cnt / sp_off (then sp_ready); after the fold stream a packs the
    // flagged segments into sp_bgr / sp_rgb (null: that output is off).  sp_s null: off.
    // lazy_tally: no wf_tally launch; the caller runs launch_tally later, when statistics are
    // asked for (the queue sizes it reads stay in the working set until the next render)
    bool lazy_tally = false;
    // dj_flags (device, kDjWords words): the b streams join stream a on the device (launch_signal /
    // launch_join) instead of through events; dj_next: the last join number handed out (the lane's,
    // advanced per join).  Null: events.
    uint64_t* dj_flags = nullptr;
    uint64_t* dj_next = nullptr;
    uint64_t* dj_err = nullptr;         // device address of the lane's page-locked error word
    hipStream_t sp_s = nullptr;
    hipEvent_t sp_cam = nullptr, sp_ready = nullptr;
    uint32_t *sp_bits = nullptr, *sp_cnt = nullptr, *sp_off = nullptr;
    uint8_t* sp_bgr = nullptr;
    float* sp_rgb = nullptr;
};
hipError_t launch_wavefront(const DevScene& sc, const FrameParams& fp, const WfBufs& b, int src, int src_occ,
                            bool count, const WfStreams& ws, hipEvent_t mark, int mark_gen);
hipError_t upload_srgb_table(const double* avg255);
// wf_tally of one chunk (rays, shadow rays and per-generation queue sizes into b.totals /
// b.gen_totals) on stream s: what launch_wavefront runs at the end unless ws.lazy_tally.
hipError_t launch_tally(const FrameParams& fp, const WfBufs& b, int n_lights, int generations, hipStream_t s);
// Device-side stream join: flag words 0 .. kDjFlags-1 (one per b stream).  launch_signal stores
// n into *flag after the stream's earlier work; launch_join waits until flag i >= n for every
// bit i of mask, or sets *err (a page-locked host word) after 2 s and goes on.
constexpr int kDjFlags = 4, kDjWords = 8;
hipError_t launch_signal(uint64_t* flag, uint64_t n, hipStream_t s);
hipError_t launch_join(uint64_t* flags, uint32_t mask, uint64_t n, uint64_t* err, hipStream_t s);
// Sparse host copies (tuning sparse_out): pixels per row segment; after the camera pass
// (b.mark set) segbits / rowcnt / rowoff of the chunk's rows (wf_chain_segs + wf_row_scan);
// after the fold the flagged segments packed in row order (wf_chain_pack).
constexpr uint32_t kSegPx = 16;
hipError_t launch_chain_segs(const FrameParams& fp, const WfBufs& b, uint32_t* segbits, uint32_t* rowcnt, uint32_t* rowoff,
                             hipStream_t s);
hipError_t launch_chain_pack(const FrameParams& fp, const uint32_t* segbits, const uint32_t* rowoff, uint8_t* pk_bgr,
                             float* pk_rgb, hipStream_t s);
// rt_ctx_reserve: a no-op launch of `workgroups` 1024-thread workgroups with private memory
// on stream s (loads trace_kernel.hip's code object, sets up the stream's queue and scratch);
// launch_path_warmup loads path_kernel.hip's.
hipError_t launch_warmup(uint32_t workgroups, hipStream_t s);
hipError_t launch_path_warmup(hipStream_t s);
// Diagnostic: div_a2(x, sphere_k(a)) and x / (2a) on the device (rt_div_a2_check).
hipError_t launch_div_a2_probe(const double* x, const double* a, uint32_t n, double* fast, double* slow, hipStream_t s);
// Diagnostic: sqrt_win(x) and sqrt(x) on the device (rt_sqrt_check).
hipError_t launch_sqrt_probe(const double* x, uint32_t n, double* fast, double* slow, hipStream_t s);

// The general path (path_kernel.hip): every material / light / camera class,
// keyed random draws, one work-item per pixel over the HBM recursion stack.
// staged: binary BVH + spheres in LDS (path_lds_bytes(sc, true) must fit).
size_t path_lds_bytes(const DevScene& sc, bool staged);
int path_waves_per_simd();          // the path kernel's occupancy (its launch bounds)
hipError_t launch_path(const DevScene& sc, const FrameParams& fp, const PathStack& st, bool staged, hipStream_t stream);

}  // namespace rtamd
