// Explicit instantiations of the observation GP's cutoff kernel for d = 9 .. 16 (obs_cutoff.h;
// split from obs_cutoff.hip so the build compiles them in parallel).
#include "obs_cutoff.h"

namespace gpmdm {
template bool launch_cut_d<9>(const CutoffParams&, hipStream_t);
template int cut_blocks_per_cu_d<9>();
template bool launch_cut_d<10>(const CutoffParams&, hipStream_t);
template int cut_blocks_per_cu_d<10>();
template bool launch_cut_d<11>(const CutoffParams&, hipStream_t);
template int cut_blocks_per_cu_d<11>();
template bool launch_cut_d<12>(const CutoffParams&, hipStream_t);
template int cut_blocks_per_cu_d<12>();
template bool launch_cut_d<13>(const CutoffParams&, hipStream_t);
template int cut_blocks_per_cu_d<13>();
template bool launch_cut_d<14>(const CutoffParams&, hipStream_t);
template int cut_blocks_per_cu_d<14>();
template bool launch_cut_d<15>(const CutoffParams&, hipStream_t);
template int cut_blocks_per_cu_d<15>();
template bool launch_cut_d<16>(const CutoffParams&, hipStream_t);
template int cut_blocks_per_cu_d<16>();
}  // namespace gpmdm
