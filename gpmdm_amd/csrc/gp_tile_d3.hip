// Explicit instantiations of the GP tile kernels for latent dimensions 9, 10, 11, 12 (split over
// translation units so the build compiles them in parallel).
#include "gp_tile.h"

namespace gpmdm {
template void launch_d<9>(const TileParams&, bool, hipStream_t);
template void launch_d<10>(const TileParams&, bool, hipStream_t);
template void launch_d<11>(const TileParams&, bool, hipStream_t);
template void launch_d<12>(const TileParams&, bool, hipStream_t);
}  // namespace gpmdm
