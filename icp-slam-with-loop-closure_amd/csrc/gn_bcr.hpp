// gn_bcr.hpp — host interface between the block-cyclic-reduction solvers
// (gn_bcr.hip: Cholesky paths, load / top kernels, dispatch; gn_bcr_gj.hip:
// the explicit-inverse levels and back-substitution).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace slamhip {

// workspace carve-up of the explicit-inverse path (nb = ceil(nv / Wb) blocks)
struct BcrGjBufs {
    double *D, *E0, *E1, *Xs, *Ys, *SP, *SN;   // nb x Wb x Wb each
    double *bz, *SPb, *SNb, *x;                // nb x Wb x mc each (mc right-hand-side columns)
};
BcrGjBufs bcr_gj_bufs(double* work, int32_t nv, int32_t Wb, int32_t mc);
int64_t bcr_gj_work_size(int32_t nv, int32_t Wb, int32_t mc);
int bcr_gj_levels(const BcrGjBufs& b, int32_t nv, int32_t Wb, int32_t mc, int32_t* status, hipStream_t st);
int bcr_gj_back(const BcrGjBufs& b, int32_t nv, int32_t Wb, int32_t mc, hipStream_t st);
// x_b of a bordered solve from the band solution Z (nv_band x mc) and the border rows BR
int bcr_border_solve(const double* Z, const double* BR, const double* rhs, const int32_t* nbr_rows, int32_t n_nbr,
                     int32_t nv_band, int32_t nbd, int32_t nvt, int32_t mc, double* xb, int32_t* status,
                     hipStream_t st);

}  // namespace slamhip
