// Second derivatives of the fused BA objectives (forward-over-reverse, dava_dual.hpp).
//
// For each problem: E, g = dE/dx, H v (v a direction per problem), dE/dobs and
// d(dE/dobs)/dx . v -- one launch, one workgroup per problem, the SAME objective
// code as the solver (ba_objective.hpp) instantiated with Dual scalars and x
// seeded with tangent v.  With an observation direction u as well (r06), the
// observations carry tangent u: the outputs become H v + (d2E/dx dobs) u and
// (d2E/dobs dx) v + (d2E/dobs2) u -- differentiating dE/dobs again.  This is the node that lets the caller differentiate
// THROUGH a solve whose error function is a fused objective: autograd's double
// backward of the reference's closure (bfgs_solver.py:133-135, create_graph)
// becomes g's VJP = H v (+ the mixed observation term).
#include "ba_objective.hpp"

namespace dava {

struct SecondArgs {
  Layout L;
  int Pv;
  const float *obs, *x, *v, *obs_v;
  const uint8_t* vis;
  float *err, *grad, *hv, *obs_grad, *obs_hv;
};

struct SecondCarve {
  int x, g, views, vpart, obsd, scratch, obs, vis_bytes_off, total_bytes;  // offsets in floats
};

__host__ __device__ inline SecondCarve carve_second(int M, int N, int Pv) {
  SecondCarve c;
  int off = 0;
  c.x = off; off += 2 * Pv;                                  // Dual
  c.g = off; off += 2 * Pv;                                  // Dual
  c.views = off; off += 2 * round_up(views_floats(M), 4);    // Dual
  c.vpart = off; off += 2 * round_up(vpart_floats(M), 4);    // Dual
  c.obsd = off; off += 2 * 2 * M * N;                        // Dual dE/dobs
  c.scratch = off; off += 2 * kWaves * 32;
  c.obs = off; off += round_up(2 * M * N, 4);
  c.vis_bytes_off = off * 4;
  c.total_bytes = c.vis_bytes_off + round_up(M * N, 16);
  return c;
}

template <int RES>
__global__ __launch_bounds__(kBlock) void ba_second_order_kernel(SecondArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const Layout L = a.L;
  const int P = L.P, M = L.M, N = L.N, MN = M * N;
  const int b = blockIdx.x, tid = threadIdx.x;
  const SecondCarve cv = carve_second(M, N, a.Pv);
  Dual* x = reinterpret_cast<Dual*>(lds + cv.x);
  Dual* g = reinterpret_cast<Dual*>(lds + cv.g);
  Dual* views = reinterpret_cast<Dual*>(lds + cv.views);
  Dual* vpart = reinterpret_cast<Dual*>(lds + cv.vpart);
  Dual* obsd = reinterpret_cast<Dual*>(lds + cv.obsd);
  float* scratch = lds + cv.scratch;
  float* obs = lds + cv.obs;
  uint8_t* vis = reinterpret_cast<uint8_t*>(lds) + cv.vis_bytes_off;
  for (int i = tid; i < a.Pv; i += kBlock) {
    x[i] = i < P ? Dual(a.x[(size_t)b * P + i], a.v ? a.v[(size_t)b * P + i] : 0.0f) : Dual(0.0f);
    g[i] = Dual(0.0f);
  }
  for (int i = tid; i < 2 * MN; i += kBlock) obs[i] = a.obs[(size_t)b * 2 * MN + i];
  for (int i = tid; i < MN; i += kBlock) vis[i] = a.vis[(size_t)b * MN + i] ? 1 : 0;
  __syncthreads();
  int buf = 0;
  Dual E(0.0f), unused(0.0f);
  ba_eval<true, false, false, false, false, RES, Dual>(L, x, nullptr, 0.0f, obs, vis, g, views, vpart, scratch, buf,
                                                       E, unused, obsd, nullptr,
                                                       a.obs_v ? a.obs_v + (size_t)b * 2 * MN : nullptr);
  if (tid == 0 && a.err) a.err[b] = E.v;
  for (int i = tid; i < P; i += kBlock) {
    if (a.grad) a.grad[(size_t)b * P + i] = g[i].v;
    if (a.hv) a.hv[(size_t)b * P + i] = g[i].t;
  }
  // dE/dobs was written per (view, point) pair by its owner thread; the eval's final
  // barrier makes it visible
  for (int i = tid; i < 2 * MN; i += kBlock) {
    if (a.obs_grad) a.obs_grad[(size_t)b * 2 * MN + i] = obsd[i].v;
    if (a.obs_hv) a.obs_hv[(size_t)b * 2 * MN + i] = obsd[i].t;
  }
}

static int second_check(const DavaScene* s) {
  if (!s) return DAVA_ERR_INVALID_ARGUMENT;
  if (s->batch < 0 || s->num_views < 2 || s->num_points < 1) return DAVA_ERR_INVALID_ARGUMENT;
  const int P = 3 + 3 * s->num_points + 6 * (s->num_views - 1) + (s->distortion ? 5 : 0);
  if (s->num_parameters != P) return DAVA_ERR_INVALID_ARGUMENT;
  if (s->batch > 0 && (!s->observations || !s->visibility)) return DAVA_ERR_INVALID_ARGUMENT;
  if (s->residual != DAVA_RESIDUAL_SQUARED_REPROJECTION && s->residual != DAVA_RESIDUAL_RAY_ANGLE)
    return DAVA_ERR_INVALID_ARGUMENT;
  if (s->residual == DAVA_RESIDUAL_RAY_ANGLE && s->distortion) return DAVA_ERR_UNSUPPORTED;
  return DAVA_OK;
}

template <int RES>
static void launch_second(const SecondArgs& a, int B, int lds, hipStream_t s) {
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(ba_second_order_kernel<RES>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL(ba_second_order_kernel<RES>, dim3(B), dim3(kBlock), lds, s, a);
}

}  // namespace dava

using namespace dava;

extern "C" int dava_ba_second_order(const DavaScene* scene, const float* x, const float* direction,
                                    float* error_out, float* grad_out, float* hv_out, float* obs_grad_out,
                                    float* obs_hv_out, void* stream) {
  return dava_ba_second_order_obs(scene, x, direction, nullptr, error_out, grad_out, hv_out, obs_grad_out, obs_hv_out,
                                  stream);
}

extern "C" int dava_ba_second_order_obs(const DavaScene* scene, const float* x, const float* direction,
                                        const float* obs_direction, float* error_out, float* grad_out, float* hv_out,
                                        float* obs_grad_out, float* obs_hv_out, void* stream) {
  const int st = second_check(scene);
  if (st != DAVA_OK) return st;
  if (scene->batch == 0) return DAVA_OK;
  if (!x) return DAVA_ERR_INVALID_ARGUMENT;
  const int Pv = round_up(scene->num_parameters, 4);
  const int lds = carve_second(scene->num_views, scene->num_points, Pv).total_bytes;
  if (lds > 160 * 1024) return DAVA_ERR_UNSUPPORTED;
  SecondArgs a;
  a.L = Layout{scene->num_views, scene->num_points, scene->num_parameters, scene->distortion ? 1 : 0};
  a.Pv = Pv;
  a.obs = scene->observations;
  a.vis = scene->visibility;
  a.x = x;
  a.v = direction;
  a.obs_v = obs_direction;
  a.err = error_out;
  a.grad = grad_out;
  a.hv = hv_out;
  a.obs_grad = obs_grad_out;
  a.obs_hv = obs_hv_out;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (scene->residual == DAVA_RESIDUAL_RAY_ANGLE) launch_second<DAVA_RESIDUAL_RAY_ANGLE>(a, scene->batch, lds, s);
  else launch_second<DAVA_RESIDUAL_SQUARED_REPROJECTION>(a, scene->batch, lds, s);
  return hipGetLastError() == hipSuccess ? DAVA_OK : DAVA_ERR_LAUNCH;
}
