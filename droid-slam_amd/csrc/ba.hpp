// Dense bundle adjustment (ba_cuda, droid_kernels.cu:1314-1434) on the GPU.
//
// Host side (ba_plan.cpp) turns the edge list of one ba() call into a static
// "plan": the depth frames kx, per-frame edge lists, the rows of the Schur
// complement per frame, and a deterministic contribution list for every
// nonzero 6x6 block of the reduced camera system.  Device side (ba_kernels.hip)
// runs every Gauss-Newton iteration with no host round trip:
//
//   ba_edge_hessian      per edge: 12x12 Hessian + 12 gradient (JtWJ, JtWr)
//   ba_frame_schur<NB>   per depth frame: C, w, Q = 1/C, E rows, and the Gram
//                        [E w]^T diag(Q) [E w] on f32 MFMA (S and S-rhs at once)
//   ba_assemble          deterministic gather of A - S into a dense fp64 matrix
//                        with the rhs appended as its last row
//   chol_dataflow        ONE persistent launch: 64x64-tile right-looking fp64
//                        Cholesky (forward solve rides along in the appended
//                        row) and the back solve, as ~3k tile tasks handed out
//                        by ticket in critical-path order and synchronised by
//                        per-tile version counters (no grid barriers)
//   ba_backsub           dz = Q (w - sum E^T dx) with the reference's t0 skip
//   ba_retract           poses <- Exp(dx) poses
#pragma once
#include <stdint.h>
#include <vector>

namespace droid {

constexpr int kHessVals = 90;      // 78 upper-tri of 12x12 + 6 vi + 6 vj
constexpr int kHessStride = 96;    // padded per (edge, split)
constexpr int kCholBlock = 64;
constexpr int kNbMax = 8;          // Gram tiles per side: 16*8 = 128 vars -> 21 rows/frame
constexpr int kLdsRow = 66;        // padded LDS row (floats) of the per-wave E image

// contribution kinds for the assembly list
enum ContribKind : int {
  kEdgeBlock = 0,   // +H12(ro+r, co+c) of edge src
  kSchurBlock = 1,  // -S_f(6*ra+r, 6*rb+c)
  kEdgeRhs = 2,     // +v12(ro+r) of edge src
  kSchurRhs = 3,    // -S_f(6*ra+r, wcol)
};

// tile tasks of the dataflow Cholesky (int4: type, i, j, k)
enum CholTaskType : int { kPotrf = 0, kTrsm = 1, kUpdate = 2, kBsolve = 3, kBupd = 4 };

struct Contrib {
  int kind, src, a0, a1;
};

struct BaPlan {
  // problem
  int E = 0, N = 0, H = 0, W = 0, HW = 0;
  int t0 = 0, t1 = 0, P = 0, K = 0, n = 0;  // n = 6P
  int motion_only = 0, eta_rows = 0;
  int nsplit = 1;        // pixel splits per edge in ba_edge_hessian
  int group_per_wave = 1;
  int nchunk = 1;        // workgroups per frame in ba_frame_schur
  int nb_max = 1;
  // host arrays (all int32)
  std::vector<int> ii, jj;              // E
  std::vector<int> kx;                  // K
  std::vector<int> f_eptr, f_edges;     // K+1, E (edges grouped by source frame)
  std::vector<int> f_rptr, r_pose, r_edge;  // K+1, R, R
  std::vector<int> f_nb, f_goff;        // K, K (float offset of Gram partials)
  std::vector<int> blk_a, blk_b, blk_cptr;  // nblk, nblk, nblk+1
  std::vector<int> rhs_cptr;            // P+1
  std::vector<Contrib> contrib, rhs_contrib;
  long gram_floats = 0;
  // reduced system: (n+1) rows of ld doubles (ld = n+1 rounded up to 8: 64-B rows)
  int ld = 0;
  // dataflow Cholesky
  int nbc = 0, nbr = 0;                 // pivot column blocks, row blocks (incl. the rhs row)
  std::vector<int> tasks;               // 4 ints per task, in ticket order
  int ntasks = 0;
  size_t sync_bytes = 0;                // ticket, abort, tile versions, y versions, x flags
  // device layout (byte offsets into the workspace)
  size_t off_ints = 0, off_hpart = 0, off_gram = 0, off_qw = 0, off_M = 0, off_x = 0,
         off_flag = 0, off_sync = 0, off_linv = 0, off_ybuf = 0, total = 0;
  // offsets (in ints) of each int array inside the int section
  size_t o_ii, o_jj, o_kx, o_feptr, o_fedges, o_frptr, o_rpose, o_redge, o_fnb, o_fgoff,
      o_blka, o_blkb, o_blkcptr, o_rhscptr, o_contrib, o_rhscontrib, o_tasks;
  std::vector<int> ints;  // packed int section, uploaded once
  bool uploaded = false;
  void* uploaded_to = nullptr;
};

// dataflow Cholesky task list for an n-pivot augmented system (ba_plan.cpp)
void build_chol_tasks(int n, int& nbc, int& nbr, std::vector<int>& tasks);

}  // namespace droid
