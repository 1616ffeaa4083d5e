// Explicit instantiations of the GP tile kernels for latent dimensions 5, 6, 7, 8 (split over
// translation units so the build compiles them in parallel).
#include "gp_tile.h"

namespace gpmdm {
template void launch_d<5>(const TileParams&, bool, hipStream_t);
template void launch_d<6>(const TileParams&, bool, hipStream_t);
template void launch_d<7>(const TileParams&, bool, hipStream_t);
template void launch_d<8>(const TileParams&, bool, hipStream_t);
}  // namespace gpmdm
