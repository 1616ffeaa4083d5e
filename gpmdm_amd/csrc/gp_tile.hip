// Dispatch of the fused GP tile kernel (gp_tile.h) on the latent dimension.  The kernels
// are instantiated in gp_tile_d*.hip.
#include "common.h"

namespace gpmdm {

template <int DI>
void launch_d(const TileParams& p, bool dyn, hipStream_t stream);

void launch_gp_tile(const TileParams& p, int d, bool dyn, hipStream_t stream) {
  if (p.n_j_max <= 0 || p.tiles_ub <= 0) return;
  switch (d) {
#define GPMDM_D(n) case n: launch_d<n>(p, dyn, stream); break;
    GPMDM_D(1) GPMDM_D(2) GPMDM_D(3) GPMDM_D(4) GPMDM_D(5) GPMDM_D(6) GPMDM_D(7) GPMDM_D(8)
    GPMDM_D(9) GPMDM_D(10) GPMDM_D(11) GPMDM_D(12) GPMDM_D(13) GPMDM_D(14) GPMDM_D(15) GPMDM_D(16)
    GPMDM_D(24) GPMDM_D(32)
#undef GPMDM_D
    default: break;  // rejected by the host (d must be 1..16, 24 or 32)
  }
}

}  // namespace gpmdm
