// tuning.h — every compile-time knob of the kernels, with its shipped default and the
// measurement behind it.  Experiment builds override them with -D
// (csrc/Makefile `variant`, tools/ab.sh); none of them changes a result — only the launch
// geometry, occupancy and schedule.  Included by wavefront.h, so every source sees one set.
#pragma once

// ---- live lists
#ifndef XRT_MAX_PARTS
#define XRT_MAX_PARTS 1024   // live-list partitions at most (per-segment schedules; C3/C4/C5 -8%..-20% vs 64)
#endif
#ifndef XRT_PART_MIN
#define XRT_PART_MIN 512     // ... of at least this many slots each (the merged schedules: 2048, at most 256)
#endif

// ---- merged schedules (k_step_merged): slots-per-wave layout by live slots (C2)
#ifndef XRT_LIVE32
#define XRT_LIVE32 90000     // below: 16 slots per wave (4 lanes each), above: 32
#endif
#ifndef XRT_LIVE8
#define XRT_LIVE8 0          // below (and above XRT_LIVE16): 8 slots per wave (8 lanes each; group traces only)
#endif
#ifndef XRT_LIVE16
#define XRT_LIVE16 20000     // below: 4 slots per wave (16 lanes each; group traces only)
#endif
#ifndef XRT_MERGED_CAMLIST
#define XRT_MERGED_CAMLIST 0 // k_step_merged: camera rays from the pixel's camera list, not the trace (C2 1 GPU
                             // 71.1 -> 71.7 ms, 8 shards 23.8 -> 23.9: -1.6% VALU, +8 spilled VGPRs); k_step_spec always
#endif
#ifndef XRT_TRACE_TLIM
#define XRT_TRACE_TLIM 1     // merged_trace: cull objects beyond the ray's closest hit so far / after occlusion (C2 -1.2%)
#endif
#ifndef XRT_STEP_WAVES
#define XRT_STEP_WAVES 4     // min waves per SIMD of k_step_merged / k_step (<= 128 VGPRs; 3 or 5: C2 -5% / -9%)
#endif
#ifndef XRT_KSTEP_LDS_REFILL
#define XRT_KSTEP_LDS_REFILL 2   // k_step in-line refill staged through LDS: 1 always, 2 except sphere-BVH scenes, 0 never
#endif
#ifndef XRT_KSTEP_512
#define XRT_KSTEP_512 0      // C3: k_step in 512-thread blocks (one LDS copy per 8 waves): -2% 1 GPU, -9% 8 shards
#endif
#ifndef XRT_KSTEP_WAVES
#define XRT_KSTEP_WAVES XRT_STEP_WAVES   // k_step (C3, C5) alone
#endif

// ---- pixel-parallel sample chains (k_pixel: Direct / Normal, pixel.hip)
#ifndef XRT_PIX_BLOCK
#define XRT_PIX_BLOCK 512    // threads per block (8 waves share one LDS copy of the scene)
#endif
#ifndef XRT_PIX_STRIDE4
#define XRT_PIX_STRIDE4 1    // k_pixel (Direct, one light): 4-word candidate stride after a window of surface hits
#endif
#ifndef XRT_PIX_GLOBAL_BVH
#define XRT_PIX_GLOBAL_BVH 1 // k_pixel reads the sphere BVH from global memory, not an LDS copy per block (C3 -1.7%)
#endif
#ifndef XRT_PIX_DEFER_BLOCK
#define XRT_PIX_DEFER_BLOCK 1024  // k_pixel threads per block, deferred-shading (C3) kernels (640 at 5 waves: C3 +18%)
#endif
#ifndef XRT_PIX_WAVES
#define XRT_PIX_WAVES 4      // min waves per SIMD (<= 128 VGPRs; 5 with 640-thread blocks: C3 +18%)
#endif
#ifndef XRT_PIX_FRUSTUM_MAX
#define XRT_PIX_FRUSTUM_MAX 8192   // sphere scenes up to this size: per-pixel camera-frustum sphere lists (0: off)
#endif
#ifndef XRT_PIX_DEFER
#define XRT_PIX_DEFER 1      // Direct on sphere scenes: queue the surface hits, shade three windows' worth at once
#endif
#ifndef XRT_PIX_SHADOW_LIST
#define XRT_PIX_SHADOW_LIST 1   // Direct, sphere scenes, one light: per-pixel shadow-ray occluder lists
#endif
#ifndef XRT_PIX_BLOCKS
#define XRT_PIX_BLOCKS 1     // k_pixel list scans skip 64-sphere blocks whose ball misses (KParams::sblk)
#endif
#ifndef XRT_PIX_PACKET
#define XRT_PIX_PACKET 1     // traces walk the scene once per wave (coherent rays), not once per lane
#endif

// ---- the fused two-level schedule (k_step_merged<..., BVH = true>: C4)
#ifndef XRT_BVH_WAVES
#define XRT_BVH_WAVES 4      // 4 waves per SIMD (128 VGPRs, ~30 spilled): C4 -11% vs 3 (no spills), 2: +40%
#endif
#ifndef XRT_BVH_LIVE64
#define XRT_BVH_LIVE64 750000   // live slots above which two-level scenes take 64 slots per wave
#endif
#ifndef XRT_BVH_LIVE32
#define XRT_BVH_LIVE32 250000   // ... 32 above this, else 16 (C4 64 spp: 8 shards 21.0 -> 16.6 ms)
#endif
#ifndef XRT_BVH_LEAF
#define XRT_BVH_LEAF 4       // triangles per leaf of the triangle BVH (at most)
#endif
#ifndef XRT_BVH_LOW_LIVE
#define XRT_BVH_LOW_LIVE 0       // two-level merged kernel: below this many live slots, the XRT_BVH_LOW_WAVES build (0: never)
#endif
#ifndef XRT_BVH_LOW_WAVES
#define XRT_BVH_LOW_WAVES 3
#endif
#ifndef XRT_BVH_TOP
#define XRT_BVH_TOP 64       // top 4-wide BVH nodes kept in LDS (at most; kStepLds bounds it); 192: neutral
#endif
#ifndef XRT_DEEP_LEAF_BATCH
#define XRT_DEEP_LEAF_BATCH 1  // leaf triangles whose loads are issued together (registers vs latency; 2: more spills)
#endif
#ifndef XRT_DEEP_SPREAD
#define XRT_DEEP_SPREAD 1    // a node's overlapped leaf triangles dealt over the quad's lanes (C4 -12%)
#endif

// ---- wavefront schedule (k_shade / k_trace*, XRT_FLAG_WAVEFRONT)
#ifndef XRT_SHADE_WAVES
#define XRT_SHADE_WAVES 1    // k_shade launch bounds (131 VGPRs, 3 waves; forcing 4/5: neutral / +9%)
#endif
#ifndef XRT_DEEP_WAVES
#define XRT_DEEP_WAVES 1     // k_trace_deep4(q) launch bounds (6 or 8 waves spill: -9% / -27%)
#endif
#ifndef XRT_2A_WAVES
#define XRT_2A_WAVES 1       // k_trace_2a_coop launch bounds
#endif

#ifndef XRT_SPEC_TWIST
#define XRT_SPEC_TWIST 1     // k_step_spec twists a slot's RNG ring in-loop when its words run short
#endif
#ifndef XRT_SPEC_VISITS
#define XRT_SPEC_VISITS 80   // ... so its launches run this many visits (without: kMT / kSpecDraws = 55); 48, 64, 128, 256: slower
#endif
#ifndef XRT_SPEC_TAIL
#define XRT_SPEC_TAIL 1      // speculative starts in the 4-slot tail launches too (k_step_spec<4, 16>)
#endif

// ---- experiment builds
#ifndef XRT_PHASE_CLOCK
#define XRT_PHASE_CLOCK 0    // k_step_spec: per-phase shader-clock cycles per wave into stats words 40..47
#endif

// ---- volumetric k_step (C5)
#ifndef XRT_VPT_EVENTS
#define XRT_VPT_EVENTS 1     // one event (a trace or one collision) per loop iteration
#endif
#ifndef XRT_VPT_EV_VISITS
#define XRT_VPT_EV_VISITS 128  // ... events per slot per launch (96: C5 +1%, 150: neutral)
#endif
#ifndef XRT_VPT_EV_DRAWS
#define XRT_VPT_EV_DRAWS 4   // ... draws of an event for the refill threshold (a collision draws <= 5)
#endif
#ifndef XRT_VPT_LOW_LIVE
#define XRT_VPT_LOW_LIVE 131072   // ... live slots below which k_step runs its 2-wave build (2 waves x 1,024 SIMDs x 64)
#endif
#ifndef XRT_VPT_EV_PF
#define XRT_VPT_EV_PF 4      // ... reload the 8-word RNG window below this many words
#endif
#ifndef XRT_CORNER_GRID
#define XRT_CORNER_GRID 1    // dense media also uploaded per cell (8 corners, 32 B): C5 +4%
#endif
