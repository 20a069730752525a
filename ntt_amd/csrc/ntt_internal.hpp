// Library-internal entry points between translation units (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ntt.h"
#include "ntt_kernels.hpp"

namespace ntt {

// Four-step addressing of one local transform (PassArgs::fs and friends, ntt_kernels.hpp).
struct FsIO {
  uint32_t fs = 0;                  // FS_MAP_IN | FS_MAP_OUT | FS_IL | FS_MAP_EPI
  uint32_t il = 0;                  // Mode I: log2 of the interleave
  FsMap min{}, mout{}, mepi{};      // input, output and epilogue-index maps (PassArgs)
  const void* tw_epi = nullptr;     // final-pass twiddle table (plan_build_fs_table) or null
  bool no_scale = false;            // inverse of a single-pass plan: no n^-1 product (the caller folded
                                    // it into another table, plan_build_fs_table's scale_log)
};

// Transform(s) of `plan` from `in` (+ `in2`: first pass starts from in * in2, polymul inverse) to
// `out` with the four-step maps.  Mode I: 2^io.il interleaved transforms (batch ignored).
int plan_run_fs(ntt_plan* plan, const void* in, const void* in2, void* out, unsigned batch, bool inverse,
                const FsIO& io, hipStream_t st);
// table[a][b] = w_n^(+-(row0 + a)(col0 + b)) 2^-scale_log in the plan's epilogue format (n = the plan's
// size); 2^(log_rows + log_cols) entries of plan_table_entry_bytes() bytes.
int plan_build_fs_table(ntt_plan* plan, void* table, unsigned log_rows, unsigned log_cols, uint64_t row0,
                        uint64_t col0, bool inverse, hipStream_t st, unsigned scale_log = 0);
size_t plan_table_entry_bytes(const ntt_plan* plan);
int plan_device(const ntt_plan* plan);
// A plan for the library's own callers (the rank plan's row / column transforms, which run only
// through plan_run_fs): no second plan of 4096-element tiles (make_wide_plan).
int plan_create_internal(ntt_plan** out, int field_id, unsigned log_n, unsigned limbs64, int device);
// pass kernels that a 2^log_x-point transform takes with this plan's engine (the four-step split)
unsigned plan_passes_for(const ntt_plan* plan, unsigned log_x);
// the largest pass radix (log2) of that transform's schedule
unsigned plan_max_radix_for(const ntt_plan* plan, unsigned log_x);

}  // namespace ntt
