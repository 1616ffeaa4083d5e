// Explicit instantiations of the GP tile kernels for latent dimensions 1, 2, 3, 4 (split over
// translation units so the build compiles them in parallel).
#include "gp_tile.h"

namespace gpmdm {
template void launch_d<1>(const TileParams&, bool, hipStream_t);
template void launch_d<2>(const TileParams&, bool, hipStream_t);
template void launch_d<3>(const TileParams&, bool, hipStream_t);
template void launch_d<4>(const TileParams&, bool, hipStream_t);
}  // namespace gpmdm
