// launch.h — host-callable kernel launchers (defined in wavefront.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "wavefront.h"

namespace xrt {
// Experiment switches (tools/*.sh) are read from the environment only in builds made with
// -DXRT_EXPERIMENTS (csrc/Makefile `variant`); the shipped library never reads them.
#ifdef XRT_EXPERIMENTS
inline const char* exp_env(const char* name) { return std::getenv(name); }
#else
inline const char* exp_env(const char*) { return nullptr; }
#endif
hipError_t launch_seed(const KParams& P, uint32_t* list, uint32_t* count, uint32_t* count_other,
                       uint32_t* req_count, hipStream_t st);
// twist the rings of the slots on P.req (count at *count); clears *zero_count
hipError_t launch_refill(const KParams& P, const uint32_t* count, uint32_t* zero_count, hipStream_t st);
hipError_t launch_trace_2a_coop(const KParams& P, const uint32_t* list, const uint32_t* count, uint32_t* zero,
                                uint32_t blocks, hipStream_t st);
// zero_deep: clear the two-level trace's queue counters first (false when the k_shade that
// precedes this trace in the render loop has cleared them)
hipError_t launch_trace(const KParams& P, const uint32_t* list, const uint32_t* count, uint32_t* zero,
                        uint32_t blocks, hipStream_t st, bool zero_deep = true);
// phase B of a two-level trace (the BVH walk of the rays launch_trace queued); no-op otherwise
hipError_t launch_trace_deep(const KParams& P, hipStream_t st);
hipError_t launch_shade(const KParams& P, const uint32_t* list, const uint32_t* count, uint32_t* out,
                        uint32_t* out_count, uint32_t* req_count, uint32_t blocks, hipStream_t st);
// fused schedule (k_step): LDS bytes it needs for this scene, 0 = scene too large for it
size_t step_lds_bytes(const KParams& P);
bool use_step_tri(const KParams& P);   // triangle scene: k_step_tri (cooperative traces)
// pixel-parallel sample chains (pixel.hip): Direct / Normal scenes that fit the LDS scene
// carve; one launch renders every pixel of the shard (after k_seed, before k_finish), taking
// pixels from the counter at `work` (zeroed by the launcher)
bool use_pixel(const KParams& P);
size_t pix_lds_bytes(const KParams& P);
hipError_t launch_pixel(const KParams& P, uint32_t* work, hipStream_t st);
// up to `visits` path segments per live slot; appends survivors to out (partitioned
// counters out_count); twists the rings of slots that ran low in-line; clears zero
// (next-next round).  req_count is unused by the step kernels (kept in the signature of
// every schedule's step launch; only the seeding k_refill reads the request list)
// dP: device copy of P (the triangle-scene kernel reads its parameters from memory)
hipError_t launch_step(const KParams& P, const KParams* dP, const uint32_t* list, const uint32_t* count, uint32_t* out,
                       uint32_t* out_count, uint32_t* zero, uint32_t* req_count, uint32_t visits, uint32_t blocks,
                       uint64_t live, hipStream_t st);
// merged-trace triangle schedule (step_tri.hip): eligibility, RNG words one segment may
// draw, LDS bytes, the per-object kernel-argument records, and the launch (same list /
// counter contract as launch_step)
bool use_step_merged(const KParams& P);
bool use_step_bvh(const KParams& P);     // two-level scenes: the merged kernel with the wave's BVH walk
uint32_t step_merged_draws(const KParams& P);
uint32_t step_merged_spw(const KParams& P, uint64_t live);   // slots per wave for `live` live slots
uint32_t step_merged_group(const KParams& P, uint32_t spw);  // lanes per slot in group traces (1 = none)
size_t step_merged_lds_bytes(const KParams& P);
void build_step_objs(const DObjBox* boxes, const DObjPlane* planes, int n, StepObjs& SO);
hipError_t launch_step_merged(const KParams& P, const KParams* dP, const StepObjs& SO, const uint32_t* list,
                              const uint32_t* count, uint32_t* out, uint32_t* out_count, uint32_t* zero,
                              uint32_t* req_count, uint32_t visits, uint64_t live, uint32_t live_part_max,
                              hipStream_t st);
// speculative sample starts for the merged schedule's group layouts (spec.hip): eligibility,
// the per-slot camera lists (once per render, before the first speculative launch), and the
// step launch at spw = 16, 8 or 4 slots per wave (same list / counter contract as
// launch_step_merged)
bool use_step_spec(const KParams& P);
constexpr uint32_t kSpecDraws = 11;   // stream words one k_step_spec visit may read past the cursor
hipError_t launch_camlist(const KParams& P, hipStream_t st);
hipError_t launch_step_spec(const KParams& P, const KParams* dP, const uint32_t* list, const uint32_t* count,
                            uint32_t* out, uint32_t* out_count, uint32_t* zero, uint32_t visits, uint32_t part_live,
                            uint32_t spw, hipStream_t st);
// the merged schedule's refill (leaves ST_RNGREQ to the merged kernel; see step_tri.hip)
hipError_t launch_refill_merged(const KParams& P, const uint32_t* count, uint32_t* zero_count, hipStream_t st);
hipError_t launch_finish(const KParams& P, hipStream_t st);
// Scene::intersect / occluded for n = P.n_slots caller rays (xrt_query): rays [n][6] on the
// device, tmax [n] or null; list / count (one partition) / zero are scratch
hipError_t launch_query(const KParams& P, const float* rays, const float* tmax, int mode, uint32_t* list,
                        uint32_t* count, uint32_t* zero, xrt_hit* out, hipStream_t st);
hipError_t launch_test_rng(const uint32_t* seeds, uint32_t n_seeds, uint32_t skip, uint32_t n, float* out,
                           uint32_t* rings, hipStream_t st);
hipError_t launch_test_trig(const float* x, uint32_t n, float* out, hipStream_t st);
hipError_t launch_test_trig_domain(uint32_t first, uint32_t count, float* s, float* c, float* r, hipStream_t st);
hipError_t launch_test_logexp(const float* x, uint32_t n, float* out, hipStream_t st);
hipError_t launch_test_powf(const float* x, uint32_t n, float y, float* out, hipStream_t st);
// Image::gammaCorrection + writePPM quantisation of n floats into n bytes
hipError_t launch_tonemap(const float* rgb, uint32_t n, float inv_gamma, uint8_t* out, hipStream_t st);
hipError_t launch_test_fastdiv(uint32_t mode, float c, float rc, uint32_t first, uint32_t count,
                               unsigned long long* nbad, uint32_t* bad, hipStream_t st);
}  // namespace xrt
