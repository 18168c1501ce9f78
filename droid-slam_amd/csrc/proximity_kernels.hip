// Proximity factors on the device: FactorGraph.add_proximity_factors
// (droid_slam/factor_graph.py:305-369) after the frame distances
// (droid_frame_distance) - the candidate mask, the NMS suppression around the
// graph's edges, the static neighbour edges, the sort by distance and the
// greedy accept-and-suppress walk - so the global backend's edge rebuild never
// round-trips a (t - t0) x (t - t1) matrix through the host or walks it in
// Python.
//
// Reference semantics kept exactly (tests/test_gpu_proximity.py checks the edge
// lists against fixtures produced by the reference's own function):
//   * candidate (i, j), i in [t0, t), j in [t1, t), index (i - t0) (t - t1) + (j - t1);
//     d = inf where i - rad < j or d > 100 (factor_graph.py:316-317);
//   * every edge of ii|ii_bad|ii_inac suppresses the L1 diamond of radius
//     max(min(|i - j| - 2, nms), 0) around it, clipped to the grid (:319-330);
//   * the static edges (i, i) [stereo] and (i, j), (j, i) for j in
//     [max(i - rad - 1, 0), i) set their own index to inf - with Python's
//     negative-index wrap when j < t1 (:333-341);
//   * candidates are visited in ascending distance (stable, NaN last, as
//     torch.argsort puts them); one with d > thresh is skipped, NaN is not (the
//     comparison is false); the walk stops when the edge list would exceed
//     max_factors (the caller turns that into n_cap accepted pairs); every
//     accepted pair suppresses its own diamond for the candidates after it (:343-366).
// The greedy walk is one wave: 64 consecutive candidates per step, accepted in
// order by a ballot loop (a pair is killed by an earlier accepted pair of the
// same step whose diamond covers it), the suppression map in global memory
// (agent-scope release stores / acquire loads, so the next step sees them).
#include "common.hpp"

#include <hipcub/hipcub.hpp>

namespace droid {

struct ProxGrid {
  int t0, t1, t, ncol, nrow;
  long n;   // nrow * ncol
};

__global__ void __launch_bounds__(256) prox_keys_kernel(const float* __restrict__ d, ProxGrid g, int rad,
                                                        float* __restrict__ keys, int* __restrict__ vals,
                                                        int* __restrict__ sup) {
  const long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= g.n) return;
  const int i = g.t0 + (int)(k / g.ncol), j = g.t1 + (int)(k % g.ncol);
  float v = d[k];
  if (i - rad < j || v > 100.0f) v = __int_as_float(0x7f800000);
  if (v != v) v = __int_as_float(0x7fc00000);   // one NaN (positive): sorted after +inf
  keys[k] = v;
  vals[k] = (int)k;
  sup[k] = 0;
}

__device__ __forceinline__ int prox_lim(int i, int j, int nms) { return max(min(abs(i - j) - 2, nms), 0); }

// thread = (edge, diamond offset)
__global__ void __launch_bounds__(256) prox_suppress_kernel(const int* __restrict__ ei, const int* __restrict__ ej,
                                                            int ne, int nms, ProxGrid g, float* __restrict__ keys) {
  const int side = 2 * nms + 1;
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (long)ne * side * side) return;
  const int e = (int)(q / (side * side)), o = (int)(q % (side * side));
  const int di = o / side - nms, dj = o % side - nms;
  const int i = ei[e], j = ej[e];
  if (abs(di) + abs(dj) > prox_lim(i, j, nms)) return;
  const int i1 = i + di, j1 = j + dj;
  if (i1 >= g.t0 && i1 < g.t && j1 >= g.t1 && j1 < g.t)
    keys[(long)(i1 - g.t0) * g.ncol + (j1 - g.t1)] = __int_as_float(0x7f800000);
}

// thread = (row i, slot): slot 0 the stereo edge (i, i), slot 1 + m the edge (i, max(i-rad-1,0) + m)
__global__ void __launch_bounds__(256) prox_static_kernel(ProxGrid g, int rad, int stereo, float* __restrict__ keys) {
  const int slots = rad + 2;
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (long)g.nrow * slots) return;
  const int i = g.t0 + (int)(q / slots), s = (int)(q % slots);
  int j;
  if (s == 0) {
    if (!stereo) return;
    j = i;
  } else {
    j = max(i - rad - 1, 0) + s - 1;
    if (j >= i) return;
  }
  long idx = (long)(i - g.t0) * g.ncol + (j - g.t1);
  if (idx < 0) idx += g.n;                   // Python's negative index
  if (idx >= 0 && idx < g.n) keys[idx] = __int_as_float(0x7f800000);
}

__global__ void __launch_bounds__(64) prox_greedy_kernel(const float* __restrict__ keys, const int* __restrict__ vals,
                                                         ProxGrid g, float thresh, int nms, int n_cap, int* sup,
                                                         int* __restrict__ out_i, int* __restrict__ out_j,
                                                         int* __restrict__ out_count) {
  const int lane = threadIdx.x;
  const long N = g.n;
  // candidates: the sorted prefix with key <= thresh, then the NaN suffix
  long lo = 0, hi = N;
  while (lo < hi) {
    const long mid = (lo + hi) >> 1;
    if (keys[mid] <= thresh) lo = mid + 1; else hi = mid;
  }
  const long n_le = lo;
  hi = N;
  while (lo < hi) {
    const long mid = (lo + hi) >> 1;
    const float v = keys[mid];
    if (v == v) lo = mid + 1; else hi = mid;
  }
  const long nan0 = lo;
  int n_acc = 0;
  for (int seg = 0; seg < 2; ++seg) {
    const long b0 = seg ? nan0 : 0, b1 = seg ? N : n_le;
    for (long base = b0; base < b1 && n_acc < n_cap; base += 64) {
      const long k = base + lane;
      bool live = false;
      int i = 0, j = 0, lim = 0;
      if (k < b1) {
        const int idx = vals[k];
        i = g.t0 + idx / g.ncol;
        j = g.t1 + idx % g.ncol;
        lim = prox_lim(i, j, nms);
        live = __hip_atomic_load(sup + idx, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0;
      }
      unsigned long long alive = __ballot(live), acc = 0;
      while (alive) {
        const int L = __ffsll((long long)alive) - 1;
        acc |= 1ull << L;
        const int iL = __shfl(i, L), jL = __shfl(j, L), lL = __shfl(lim, L);
        alive &= ~__ballot(abs(i - iL) + abs(j - jL) <= lL);
        alive &= ~(1ull << L);
      }
      int nacc = __popcll(acc);
      if (n_acc + nacc > n_cap) {   // the edge list is full: keep the first ones in order
        unsigned long long keep = 0;
        for (int r = 0; r < n_cap - n_acc; ++r) {
          const int L = __ffsll((long long)(acc & ~keep)) - 1;
          keep |= 1ull << L;
        }
        acc = keep;
        nacc = n_cap - n_acc;
      }
      if ((acc >> lane) & 1ull) {
        const int r = n_acc + __popcll(acc & ((1ull << lane) - 1ull));
        out_i[r] = i;
        out_j[r] = j;
        for (int di = -lim; di <= lim; ++di)
          for (int dj = -(lim - abs(di)); dj <= lim - abs(di); ++dj) {
            const int i1 = i + di, j1 = j + dj;
            if (i1 >= g.t0 && i1 < g.t && j1 >= g.t1 && j1 < g.t)
              __hip_atomic_store(sup + (long)(i1 - g.t0) * g.ncol + (j1 - g.t1), 1, __ATOMIC_RELEASE,
                                 __HIP_MEMORY_SCOPE_AGENT);
          }
      }
      n_acc += nacc;
    }
  }
  if (lane == 0) out_count[0] = n_acc;
}

struct ProxWs {
  size_t keys, vals, keys2, vals2, sup, temp, temp_bytes, total;
};

static ProxWs prox_layout(long n) {
  ProxWs w{};
  size_t temp_bytes = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, (const float*)nullptr, (float*)nullptr,
                                         (const int*)nullptr, (int*)nullptr, (int)n) != hipSuccess)
    temp_bytes = 0;   // (a size query; droid_proximity_select reports the sort's own error)
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  w.keys = 0;
  w.vals = al(w.keys + n * 4);
  w.keys2 = al(w.vals + n * 4);
  w.vals2 = al(w.keys2 + n * 4);
  w.sup = al(w.vals2 + n * 4);
  w.temp = al(w.sup + n * 4);
  w.temp_bytes = temp_bytes;
  w.total = al(w.temp + temp_bytes);
  return w;
}

}  // namespace droid

using namespace droid;

extern "C" {

// Bytes of device workspace droid_proximity_select needs for the grid [t0, t) x [t1, t).
size_t droid_proximity_workspace(int t0, int t1, int t) {
  if (t0 < 0 || t1 < 0 || t0 >= t || t1 >= t) return 0;
  return prox_layout((long)(t - t0) * (t - t1)).total;
}

// add_proximity_factors after the distances: d = the (t - t0) x (t - t1)
// distances of video.distance(meshgrid), row-major; ei/ej = the graph's edges
// (ii|ii_bad|ii_inac, jj|...) that suppress their neighbourhoods; n_cap = how
// many candidate pairs may still be accepted before the edge list exceeds
// max_factors.  Writes the accepted pairs in acceptance order to out_i/out_j
// (capacity n_cap) and their count to *out_count (all device memory).  The
// caller prepends the static edges, which it builds itself.
int droid_proximity_select(const float* d, int t0, int t1, int t, int rad, int nms, float thresh, const int* ei,
                           const int* ej, int ne, int stereo, int n_cap, int* out_i, int* out_j, int* out_count,
                           void* ws, size_t ws_bytes, hipStream_t stream) {
  if (t0 < 0 || t1 < 0 || t0 >= t || t1 >= t || rad < 0 || nms < 0 || ne < 0 || n_cap < 0 || !d || !out_count ||
      (ne && (!ei || !ej)) || (n_cap && (!out_i || !out_j)))
    return fail(kInvalidArgument, "proximity_select: bad arguments");
  const long n = (long)(t - t0) * (t - t1);
  if (n >= 0x7fffffffL) return fail(kUnsupported, "proximity_select: grid too large");
  const ProxWs w = prox_layout(n);
  if (!ws || ws_bytes < w.total) return fail(kInvalidArgument, "proximity_select: workspace too small");
  char* base = static_cast<char*>(ws);
  float* keys = reinterpret_cast<float*>(base + w.keys);
  int* vals = reinterpret_cast<int*>(base + w.vals);
  float* keys2 = reinterpret_cast<float*>(base + w.keys2);
  int* vals2 = reinterpret_cast<int*>(base + w.vals2);
  int* sup = reinterpret_cast<int*>(base + w.sup);
  ProxGrid g{t0, t1, t, t - t1, t - t0, n};
  prox_keys_kernel<<<(unsigned)(n + 255) / 256, 256, 0, stream>>>(d, g, rad, keys, vals, sup);
  DROID_LAUNCH_CHECK();
  const long nsup = (long)ne * (2 * nms + 1) * (2 * nms + 1);
  if (nsup > 0) {
    prox_suppress_kernel<<<(unsigned)(nsup + 255) / 256, 256, 0, stream>>>(ei, ej, ne, nms, g, keys);
    DROID_LAUNCH_CHECK();
  }
  const long nst = (long)g.nrow * (rad + 2);
  prox_static_kernel<<<(unsigned)(nst + 255) / 256, 256, 0, stream>>>(g, rad, stereo, keys);
  DROID_LAUNCH_CHECK();
  size_t tb = w.temp_bytes;
  DROID_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(base + w.temp, tb, keys, keys2, vals, vals2, (int)n, 0,
                                                     32, stream));
  prox_greedy_kernel<<<1, 64, 0, stream>>>(keys2, vals2, g, thresh, nms, n_cap, sup, out_i, out_j, out_count);
  DROID_LAUNCH_CHECK();
  return kOk;
}

}  // extern "C"
