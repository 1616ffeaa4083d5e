// Explicit instantiations of the GP tile kernels for latent dimensions 24, 32 (split over
// translation units so the build compiles them in parallel).
#include "gp_tile.h"

namespace gpmdm {
template void launch_d<24>(const TileParams&, bool, hipStream_t);
template void launch_d<32>(const TileParams&, bool, hipStream_t);
}  // namespace gpmdm
