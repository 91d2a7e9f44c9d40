// esgpu_collect_inst.hip — instantiates the collect kernels of one (ORD, HK, MET) triple (-DESGPU_INST_ORD,
// -DESGPU_INST_HK, -DESGPU_INST_MET); the Makefile builds this file once per triple so the ~80 kernel variants compile
// in parallel.
#include "esgpu_collect.hpp"

#if !defined(ESGPU_INST_ORD) || !defined(ESGPU_INST_HK) || !defined(ESGPU_INST_MET)
#error "ESGPU_INST_ORD / ESGPU_INST_HK / ESGPU_INST_MET select the instantiation"
#endif

namespace esgpu {

template <bool ORD, int HK, int MET>
void launch_collect_met(const CollectParams& p, bool wide, uint32_t grid, size_t lds, hipStream_t st) {
    launch_t<ORD, HK, MET>(p, wide, grid, lds, st);
}
template <bool ORD, int HK, int MET>
int collect_occ_met(size_t lds, int vk, bool wide) {
    return occ_t<ORD, HK, MET>(lds, vk, wide);
}

template void launch_collect_met<(bool)ESGPU_INST_ORD, ESGPU_INST_HK, ESGPU_INST_MET>(const CollectParams&, bool, uint32_t, size_t,
                                                                                       hipStream_t);
template int collect_occ_met<(bool)ESGPU_INST_ORD, ESGPU_INST_HK, ESGPU_INST_MET>(size_t, int, bool);

}  // namespace esgpu
