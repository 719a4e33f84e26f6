// mpc_structure.hpp -- recognises the stage structure of mpcPlanner's QPs in a generic CSC
// pattern and builds the shared tables of the one-QP-per-wavefront kernel (mpc_wave.hpp).
//
// The reference's variable order (mpcPlanner.cpp:491,501) is all states x_0..x_{N-1} (8 each)
// followed by all controls u_0..u_{N-2} (5 each).  In "stage order" v' = 13k + r, stage k holds
// x_k (r < 8) and u_k (8 <= r < 13); the last stage holds x_{N-1} only.  The classifier accepts a
// pattern when
//   * n = 13N - 5, P is diagonal (castMPCToQPHessian, :932-951),
//   * every variable has a single-entry ("box") row (the identity block, :1023-1026),
//   * every other ("general") row has <= 4 entries that lie in one stage k plus, optionally,
//     the state part x_{k+1} of the next stage (dynamics rows :994-1020, FOV half-spaces
//     :1027-1038, obstacle rows :1052-1069).
// Then M = P + sigma I + A' R A is block tridiagonal over stages with an 8-wide coupling, which
// the wave kernel factors stage by stage.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace impc {

struct MpcStructure {
    int32_t n = 0, m = 0, N = 0, W = 0, mg = 0, CG = 0, nnzP = 0, nnzA = 0;
    int32_t max_general_per_stage = 0;
    std::vector<int32_t> var_orig, var_pdiag, var_boxrow, var_boxpos;  // [n], stage order
    std::vector<int32_t> gen_row;                                      // [mg]
    std::vector<int32_t> gen_col, gen_pos;                             // [4 mg], stage-order col / CSC slot, -1 pad
    std::vector<int32_t> colg;                                         // [n * CG] entry ids g*4+e, -1 pad
    // products buffer of the structured kernel (mpc_wave.hpp): every column has kProdTier1 slots
    // in the first tier; the HS columns with more general entries ("heavy": the positions and the
    // slack of a stage with obstacle rows) continue in a second tier, at their index col_hid
    int32_t HS = 0;
    std::vector<int32_t> col_hid;                                      // [n], -1 for light columns
    std::vector<int32_t> term_ptr, term;                               // factorisation assembly program
    // Returns "" when the pattern is stage-structured, else the reason it is not.
    std::string analyse(int64_t n, int64_t m, const int64_t *Pp, const int64_t *Pi, const int64_t *Ap,
                        const int64_t *Ai);
};

constexpr int kStageDests = 13 * 13 + 8 * 13;  // M_kk (13x13) + coupling B_k (8x13)
constexpr int kProdTier1 = 4;                  // first-tier product slots per column

}  // namespace impc
