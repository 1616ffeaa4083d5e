// Explicit instantiations of the GP tile kernels for latent dimensions 13, 14, 15, 16 (split over
// translation units so the build compiles them in parallel).
#include "gp_tile.h"

namespace gpmdm {
template void launch_d<13>(const TileParams&, bool, hipStream_t);
template void launch_d<14>(const TileParams&, bool, hipStream_t);
template void launch_d<15>(const TileParams&, bool, hipStream_t);
template void launch_d<16>(const TileParams&, bool, hipStream_t);
}  // namespace gpmdm
