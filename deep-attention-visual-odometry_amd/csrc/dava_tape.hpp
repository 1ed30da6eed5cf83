// Layout of the solve tape: what a recording fused solve (dava_ba_solve_record) keeps in HBM so
// that the adjoint kernel (bfgs_adjoint.hip) can run the solve backwards -- the reference's
// differentiate-through-the-solve mode (bfgs_solver.py:85, :134, :213-215) without a dense
// (B, P, P) inverse Hessian per iteration in an autograd graph.
//
// Per problem b, K = iterations, kcap = max(K - 1, 1), Pv = P rounded up to 4, all fp32:
//   hist   (B, 2, kcap, Pv)  history rows S[j] = s_j, W[j] = w_j = H_j' y_{j+1} (the compact
//                            inverse-Hessian state, every entry in HBM -- no LDS-resident ones)
//   x      (B, K, Pv)        x_k at the start of iteration k
//   g      (B, K, Pv)        g_k = dE/dx (x_k)
//   scal   (B, T)            [alpha_0..alpha_{K-1} | rho_0..rho_{K-1} | c_0..c_{K-1} | gamma],
//                            T = round_up(3 K + 1, 4)
//   vecs   (B, V)            global-vector-mode recordings only: the solve's O(P) vectors (V floats per
//                            problem, scratch of the recording launch; the adjoint does not read them)
//   queue  256 bytes          the work-queue counter of the recording launch
#pragma once

#include <stddef.h>

namespace dava {

struct TapeLayout {
  int K, kcap, Pv, T;
  size_t hist, x, g, scal, vecs;  // offsets in floats
  size_t queue_byte, total_bytes;
};

inline int tape_round_up(int v, int m) { return (v + m - 1) / m * m; }

inline TapeLayout tape_layout(int B, int P, int K, int vec_floats = 0) {
  TapeLayout t;
  t.K = K > 0 ? K : 1;
  t.kcap = K > 1 ? K - 1 : 1;
  t.Pv = tape_round_up(P, 4);
  t.T = tape_round_up(3 * t.K + 1, 4);
  const size_t b = (size_t)(B > 0 ? B : 0);
  t.hist = 0;
  t.x = t.hist + b * 2 * (size_t)t.kcap * t.Pv;
  t.g = t.x + b * (size_t)t.K * t.Pv;
  t.scal = t.g + b * (size_t)t.K * t.Pv;
  t.vecs = t.scal + b * (size_t)t.T;
  t.queue_byte = (t.vecs + b * (size_t)(vec_floats > 0 ? vec_floats : 0)) * sizeof(float);
  t.total_bytes = t.queue_byte + 256;
  return t;
}

}  // namespace dava
