/*
 * dmf_diag.h — diagnostic, A/B and test controls of libdmf.so (not the product ABI).
 *
 * Nothing here changes a result: every fusion kernel and every knob value gives the same
 * integer counters, flags and lists (the GPU suite checks each against the oracle) -- except
 * DMF_KNOB_FAULT_INJECT, the test hook of the device-side layout check (dmf_fuse_status).  The
 * controls are PER VOLUME (no process-global state, no environment variables read by the
 * library); a new volume starts with every control at its default.  Declared apart from
 * include/dmf.h so that callers of the product ABI never see them.
 */
#ifndef DMF_DIAG_H_
#define DMF_DIAG_H_

#include <stdint.h>

#include "dmf.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Fusion implementation of dmf_fuse_depth(_device) on this volume. */
enum dmf_fuse_variant {
  DMF_FUSE_DEFAULT = 0,    /* by grid size: DMF_FUSE_SLAB for a longest axis of 256..1024 cells, else DMF_FUSE_LDS_BOX */
  DMF_FUSE_LDS_BOX = 31,   /* k_fuse_l<12, 1280>: one wave per 8x8 pixel packet, LDS box per round */
  DMF_FUSE_CELL_WALK = 40, /* brick pipeline with the per-cell walk k_bk_fuse (24-B records): independent exact check */
  DMF_FUSE_SLAB = 57       /* brick pipeline, slab walk k_bk_fuse_s on 20-B records, at any grid <= 1024 cells/axis */
};
int dmf_fuse_set_variant(dmf_volume* v, int32_t variant);
int dmf_fuse_get_variant(const dmf_volume* v, int32_t* variant);
/* Name of the (dominant) fusion kernel this volume's latest fusion call launched; before
 * any call, the kernel its variant uses on a 512^3 grid. */
const char* dmf_fuse_kernel_name(const dmf_volume* v);

/* Tuning / test knobs; value 0 = the default. */
enum dmf_knob {
  DMF_KNOB_SUPER_POSES = 1, /* cap of the poses per super-batch (one pass A over all of them) */
  DMF_KNOB_PAIR_CAP = 2,    /* cap of the pair records a batch may hold (must hold any one frame's pairs) */
  DMF_KNOB_BATCH_POSES = 3, /* cap of the poses per device-cut pose batch */
  DMF_KNOB_PART_MAX = 4,    /* pairs per part of phase F's queue (1024..65535; default 65535) */
  DMF_KNOB_SPAN = 5,        /* 8x8 packets per pass-A/B workgroup (4..1023) */
  DMF_KNOB_TAIL_SPLIT = 6,  /* phase F's queue tail split: -1 off, k > 0 = the last k x CUs parts quartered
                               (default: 2 for serial calls, off for pipelined ones) */
  DMF_KNOB_REVERSE_KERNEL = 7, /* reverseRayTraceFast march: 0 default (wave queues in spatial order + distance
                                  field, workgroup units from per-XCD queues: k_reverse_x), 1 plain, 2 plain +
                                  brick skip, 3 queue in insertion order, 4 per-XCD queues of wave units, 5 the
                                  spatial-order queues on a (chunk, pose) grid (k_reverse_q) */
  DMF_KNOB_FWD_SKIP = 8,    /* forward march empty-space skipping: 0 default (on), -1 off */
  DMF_KNOB_A_HASH = 9,      /* pass A's histogram: 0 default (hashed, 2048 words, above 8192 bricks; direct
                               below), -1 always direct, k > 0 always hashed with k words (rounded up to a
                               power of two, 16..16384; a workgroup whose table overflows is redone with the direct one) */
  DMF_KNOB_FAULT_INJECT = 10, /* test hook: k > 0 makes the first pair of thread 0 of every pass-B workgroup of the
                                  call's first pose take k extra slots, so that passes A and B disagree (the results are
                                  then invalid; dmf_fuse_status reports it, and no store leaves the pair
                                  buffers); 0 = off */
  DMF_KNOB_FWD_KERNEL = 11,  /* batched forward first hits (dmf_forward_first_hits_device): 0 default (a grid of
                                (tile block, pose): k_forward), 1 per-XCD unit queues (k_forward_x), 2 per-wave lane refill
                                over units of 8x8 tiles (k_forward_q) */
  DMF_KNOB_BDIST_CAP = 12,   /* saturation of the brick distance field of the reverse / forward marches' empty-space
                                jumps, in bricks (1..255; 0 = the default 63); rebuilt at the next march */
  DMF_KNOB_COUNT = 13
};
int dmf_volume_set_knob(dmf_volume* v, int32_t knob, int64_t value);
int dmf_volume_get_knob(const dmf_volume* v, int32_t knob, int64_t* value);

#ifdef __cplusplus
}
#endif
#endif /* DMF_DIAG_H_ */
