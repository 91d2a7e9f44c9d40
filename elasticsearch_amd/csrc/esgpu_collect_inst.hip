// esgpu_collect_inst.hip — instantiates the collect kernels of one (ORD, HK) pair (-DESGPU_INST_ORD, -DESGPU_INST_HK);
// the Makefile builds this file once per pair so the ~70 kernel variants compile in parallel.
#include "esgpu_collect.hpp"

#ifndef ESGPU_INST_ORD
#error "ESGPU_INST_ORD / ESGPU_INST_HK select the instantiation"
#endif

namespace esgpu {

template <bool ORD, int HK>
void launch_collect_inst(const CollectParams& p, int met, bool wide, uint32_t grid, size_t lds, hipStream_t st) {
    launch_m<ORD, HK>(p, met, wide, grid, lds, st);
}
template <bool ORD, int HK>
int collect_occ_inst(int met, size_t lds, int vk, bool wide) {
    return occ_m<ORD, HK>(met, lds, vk, wide);
}

template void launch_collect_inst<(bool)ESGPU_INST_ORD, ESGPU_INST_HK>(const CollectParams&, int, bool, uint32_t, size_t, hipStream_t);
template int collect_occ_inst<(bool)ESGPU_INST_ORD, ESGPU_INST_HK>(int, size_t, int, bool);

}  // namespace esgpu
