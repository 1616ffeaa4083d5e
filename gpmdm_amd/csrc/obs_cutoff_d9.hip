// Explicit instantiations of the observation GP's cutoff kernel for d = 9 .. 16 (obs_cutoff.h;
// split from obs_cutoff.hip so the build compiles them in parallel).
#include "obs_cutoff.h"

namespace gpmdm {
template void launch_cut_d<9>(const CutoffParams&, hipStream_t);
template void launch_cut_d<10>(const CutoffParams&, hipStream_t);
template void launch_cut_d<11>(const CutoffParams&, hipStream_t);
template void launch_cut_d<12>(const CutoffParams&, hipStream_t);
template void launch_cut_d<13>(const CutoffParams&, hipStream_t);
template void launch_cut_d<14>(const CutoffParams&, hipStream_t);
template void launch_cut_d<15>(const CutoffParams&, hipStream_t);
template void launch_cut_d<16>(const CutoffParams&, hipStream_t);
}  // namespace gpmdm
