// align_inst.hip -- instantiates the alignment kernels (align_kernels.h) for one range of query
// lengths; compiled once per part with -DALIGN_PART=p so the instantiations build in parallel.
#include "align_kernels.h"

#ifndef ALIGN_PART
#error "ALIGN_PART must be defined"
#endif

namespace uc {
#define UC_CAT2(a, b) a##b
#define UC_CAT(a, b) UC_CAT2(a, b)
void UC_CAT(fill_align_part, ALIGN_PART)(AlignFn* a) {
  AlignRange<kAlignPartLo[ALIGN_PART + 1] - 1, kAlignPartLo[ALIGN_PART]>::fill(a);
}
}  // namespace uc
