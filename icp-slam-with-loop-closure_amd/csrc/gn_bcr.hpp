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
    double* bzo;                               // nb x Wb x mc: the odd blocks' z (Schur solves)
    int32_t* ready;                            // [0]: the back-substitution's epoch (top kernel)
    uint64_t* xg;                              // nb x 2 Wb: x as tagged granules (XCD-local back-substitution)
};
// A bordered solve with the border's Schur complement accumulated during the
// elimination: the RHS block is [r_a | B] (mc
// columns); every eliminated block i listed in pslot (slot k >= 0) adds
// P_i = Y_i^T G_i Y_i (Y_i its reduced RHS block, G_i = D_i^-1) to slot k of
// P; the top kernel forms S = C - sum P[B, B] - P_0[B, B] and s = r_b - ...,
// solves x_b = S^-1 s, and the back-substitution runs on ONE column
// z_i[:, 0] - z_i[:, B] x_b.  Odd blocks write their z to bzo (their inputs
// in bz stay intact: every RHS tile of a block reads all of its columns).
struct BcrSchur {
    const int32_t* pslot;   // nb entries: P slot of block i, -1 none
    double* P;              // n_slots x mc x mc
    int32_t n_slots;
    const double* BR;       // the border rows of H (nbd x nvt, lower triangle)
    const double* rhs;      // nvt: r_b = rhs[nv_band + k]
    int32_t nv_band, nbd, nvt;
    double* xb;             // nbd: the border's solution
    int32_t* status;        // the iteration's status word (a fused wait that timed out sets 2)
};
// The XCD-local fused back-substitution on (1, default) or off (0).
void bcr_gj_set_fused(int on);
int bcr_gj_get_fused();
void bcr_gj_set_fused_wait(uint32_t ticks);   // diagnostics: the longest wait (s_memrealtime ticks)
BcrGjBufs bcr_gj_bufs(double* work, int32_t nv, int32_t Wb, int32_t mc);
int64_t bcr_gj_work_size(int32_t nv, int32_t Wb, int32_t mc);
int bcr_gj_levels(const BcrGjBufs& b, int32_t nv, int32_t Wb, int32_t mc, int32_t* status, hipStream_t st,
                  const BcrSchur* sc = nullptr);
int bcr_gj_back(const BcrGjBufs& b, int32_t nv, int32_t Wb, int32_t mc, hipStream_t st,
                const BcrSchur* sc = nullptr);
// x_b of a bordered solve from the band solution Z (nv_band x mc) and the border rows BR
int bcr_border_solve(const double* Z, const double* BR, const double* rhs, const int32_t* nbr_rows, int32_t n_nbr,
                     int32_t nv_band, int32_t nbd, int32_t nvt, int32_t mc, double* xb, int32_t* status,
                     hipStream_t st);

}  // namespace slamhip
