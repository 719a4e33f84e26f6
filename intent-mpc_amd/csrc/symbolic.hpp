// symbolic.hpp -- host-side symbolic analysis shared by every QP of a batch.
//
// OSQP 0.6.2 (osqp_setup -> init_linsys_solver, reference osqp.h:58) factors the quasi-definite
// KKT [[P + sigma I, A'], [A, -diag(1/rho)]] with AMD + QDLDL.  The batched solver instead
// factors the reduced (Schur-complement) system
//     M = P + sigma I + A' diag(rho) A          (SPD, n x n)
// whose solution gives x~ directly and z~ = A x~ -- mathematically identical to OSQP's
// KKT solve ("Reduced KKT").  Everything that depends only on the sparsity pattern is
// computed here once per batch:
//   * a fill-reducing minimum-degree ordering of M,
//   * the CSC pattern of upper(M) in factor order and an assembly program that adds
//     P, sigma and every A' R A product into it,
//   * a replay of QDLDL's up-looking LDL^T symbolic phase (etree, column counts, the exact
//     sequence of column updates) so the device executes the numeric factorisation as a
//     fixed, branch-free program,
//   * CSR views of A and L for gather-only SpMV / triangular solves.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace impc {

struct Symbolic {
    int32_t n = 0, m = 0, nnzP = 0, nnzA = 0;
    // problem pattern (CSC, original order)
    std::vector<int32_t> Pp, Pi, Ap, Ai;
    // CSR view of A: row r holds Arp[r]..Arp[r+1]; value slot in CSC, column, factor position
    std::vector<int32_t> Arp, Arpos, Arcol, Arcolf;
    // ordering: perm[k] = variable at factor position k, iperm[var] = k
    std::vector<int32_t> perm, iperm;
    // upper(M) in factor order, CSC; Mdiag[k] = slot of (k,k)
    std::vector<int32_t> Mp, Mi, Mdiag;
    // assembly: Mval[Pt_dest] += Ps[Pt_src];  Mval[At_dest] += As[At_a] * rho[At_r] * As[At_b]
    std::vector<int32_t> Pt_dest, Pt_src;
    std::vector<int32_t> At_dest, At_a, At_b, At_r;
    // L (unit lower, CSC in factor order) and its CSR view (value slot per entry)
    std::vector<int32_t> Lp, Li, Lrp, Lrc, Lrpos;
    // numeric-factorisation program (QDLDL_factor replay): for row k, updates upd_ptr[k]..
    // each = (column c, L slots [js, je) already filled in column c, slot w to write L(k,c))
    std::vector<int32_t> upd_ptr, upd_c, upd_js, upd_je, upd_w;
    int64_t nnzM = 0, nnzL = 0, n_upd = 0, factor_flops = 0;
    int32_t max_row_L = 0;

    // Returns empty string on success, else the validation error.
    std::string build(int64_t n, int64_t m, const int64_t *Pp, const int64_t *Pi, const int64_t *Ap,
                      const int64_t *Ai);
};

}  // namespace impc
