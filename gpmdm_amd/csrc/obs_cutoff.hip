// The observation GP's cutoff kernel (obs_cutoff.h): the launcher and the instantiations for
// d = 1 .. 8 (d = 9 .. 16: obs_cutoff_d9.hip, compiled in parallel).
#include "obs_cutoff.h"

namespace gpmdm {

extern template void launch_cut_d<9>(const CutoffParams&, hipStream_t);
extern template void launch_cut_d<10>(const CutoffParams&, hipStream_t);
extern template void launch_cut_d<11>(const CutoffParams&, hipStream_t);
extern template void launch_cut_d<12>(const CutoffParams&, hipStream_t);
extern template void launch_cut_d<13>(const CutoffParams&, hipStream_t);
extern template void launch_cut_d<14>(const CutoffParams&, hipStream_t);
extern template void launch_cut_d<15>(const CutoffParams&, hipStream_t);
extern template void launch_cut_d<16>(const CutoffParams&, hipStream_t);

void launch_obs_cutoff(const CutoffParams& p, int d, hipStream_t s) {
  switch (d) {
    case 1: launch_cut_d<1>(p, s); break;
    case 2: launch_cut_d<2>(p, s); break;
    case 3: launch_cut_d<3>(p, s); break;
    case 4: launch_cut_d<4>(p, s); break;
    case 5: launch_cut_d<5>(p, s); break;
    case 6: launch_cut_d<6>(p, s); break;
    case 7: launch_cut_d<7>(p, s); break;
    case 8: launch_cut_d<8>(p, s); break;
    case 9: launch_cut_d<9>(p, s); break;
    case 10: launch_cut_d<10>(p, s); break;
    case 11: launch_cut_d<11>(p, s); break;
    case 12: launch_cut_d<12>(p, s); break;
    case 13: launch_cut_d<13>(p, s); break;
    case 14: launch_cut_d<14>(p, s); break;
    case 15: launch_cut_d<15>(p, s); break;
    case 16: launch_cut_d<16>(p, s); break;
    default: break;   // refused by gpmdm_model_set_obs_cutoff
  }
}

}  // namespace gpmdm
