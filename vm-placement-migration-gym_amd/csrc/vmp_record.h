// vmp_record.h — recorder state shared by vmp_record.hip and vmp_capi.cpp.
#pragma once
#include <stdint.h>

namespace vmp {
struct RecArgs {
  uint16_t *prev;     // [N][V] previous post-step placement
  uint32_t *life_n;   // [N][V] status count of the slot's current life
  int32_t *alloc;     // [N][V] allocated_at of the current life, -1 = none
  uint32_t *waits;    // [N][V] WAIT statuses at or after allocated_at
  uint32_t *hist;     // [N][2][VMP_REC_BINS] pending, slowdown
  double *sums;       // [N][VMP_NREC]
  const int32_t *act;      // this step's actions [N][V]
  const uint8_t *valid;    // [N][V]
  const double *reward;    // [N]
};
}  // namespace vmp
