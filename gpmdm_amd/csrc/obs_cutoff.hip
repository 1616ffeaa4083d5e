// The observation GP's cutoff kernel (obs_cutoff.h): the launcher and the instantiations for
// d = 1 .. 8 (d = 9 .. 16: obs_cutoff_d9.hip, compiled in parallel).
#include "obs_cutoff.h"

#include <atomic>

namespace gpmdm {

extern template bool launch_cut_d<9>(const CutoffParams&, hipStream_t);
extern template int cut_blocks_per_cu_d<9>();
extern template bool launch_cut_d<10>(const CutoffParams&, hipStream_t);
extern template int cut_blocks_per_cu_d<10>();
extern template bool launch_cut_d<11>(const CutoffParams&, hipStream_t);
extern template int cut_blocks_per_cu_d<11>();
extern template bool launch_cut_d<12>(const CutoffParams&, hipStream_t);
extern template int cut_blocks_per_cu_d<12>();
extern template bool launch_cut_d<13>(const CutoffParams&, hipStream_t);
extern template int cut_blocks_per_cu_d<13>();
extern template bool launch_cut_d<14>(const CutoffParams&, hipStream_t);
extern template int cut_blocks_per_cu_d<14>();
extern template bool launch_cut_d<15>(const CutoffParams&, hipStream_t);
extern template int cut_blocks_per_cu_d<15>();
extern template bool launch_cut_d<16>(const CutoffParams&, hipStream_t);
extern template int cut_blocks_per_cu_d<16>();

bool launch_obs_cutoff(const CutoffParams& p, int d, hipStream_t s) {
  switch (d) {
    case 1: return launch_cut_d<1>(p, s);
    case 2: return launch_cut_d<2>(p, s);
    case 3: return launch_cut_d<3>(p, s);
    case 4: return launch_cut_d<4>(p, s);
    case 5: return launch_cut_d<5>(p, s);
    case 6: return launch_cut_d<6>(p, s);
    case 7: return launch_cut_d<7>(p, s);
    case 8: return launch_cut_d<8>(p, s);
    case 9: return launch_cut_d<9>(p, s);
    case 10: return launch_cut_d<10>(p, s);
    case 11: return launch_cut_d<11>(p, s);
    case 12: return launch_cut_d<12>(p, s);
    case 13: return launch_cut_d<13>(p, s);
    case 14: return launch_cut_d<14>(p, s);
    case 15: return launch_cut_d<15>(p, s);
    case 16: return launch_cut_d<16>(p, s);
    default: return false;   // refused by gpmdm_model_set_obs_cutoff
  }
}

int cutoff_tile_particles(int d) { return d <= 8 ? 32 : 64; }
int cutoff_tile_list_chunk() { return 32; }   // 4 waves x 8 tiles, 8 x 4 above d = 8

int cutoff_slots(int d) {
  static std::atomic<int> cache[kMaxD + 1];
  if (d < 1 || d > 16) return 1;
  int v = cache[d].load(std::memory_order_relaxed);
  if (v > 0) return v;
  int b = 1;
  switch (d) {
    case 1: b = cut_blocks_per_cu_d<1>(); break;
    case 2: b = cut_blocks_per_cu_d<2>(); break;
    case 3: b = cut_blocks_per_cu_d<3>(); break;
    case 4: b = cut_blocks_per_cu_d<4>(); break;
    case 5: b = cut_blocks_per_cu_d<5>(); break;
    case 6: b = cut_blocks_per_cu_d<6>(); break;
    case 7: b = cut_blocks_per_cu_d<7>(); break;
    case 8: b = cut_blocks_per_cu_d<8>(); break;
    case 9: b = cut_blocks_per_cu_d<9>(); break;
    case 10: b = cut_blocks_per_cu_d<10>(); break;
    case 11: b = cut_blocks_per_cu_d<11>(); break;
    case 12: b = cut_blocks_per_cu_d<12>(); break;
    case 13: b = cut_blocks_per_cu_d<13>(); break;
    case 14: b = cut_blocks_per_cu_d<14>(); break;
    case 15: b = cut_blocks_per_cu_d<15>(); break;
    case 16: b = cut_blocks_per_cu_d<16>(); break;
  }
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  v = b * cus;
  cache[d].store(v, std::memory_order_relaxed);
  return v;
}

}  // namespace gpmdm
