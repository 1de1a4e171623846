// Engine-side supernode amalgamation (1x1 grids).
//
// The reference's symbfact keeps only fundamental supernodes (T2_SUPER,
// SRC/symbfact.c:39) plus relaxed leaf subtrees, so the LUstruct pdgssvx
// hands pdgstrf for a nested-dissection ordering of a 3D stencil has ~80 %
// width-1 supernodes: every separator column with a private neighbour in an
// ancestor separator ends a supernode (100^3: 217 069 supernodes, 163 328 of
// width 1, an elimination tree 909 supernodes deep).  A right-looking
// factorization of that partition does a rank-1 Schur update per width-1
// supernode -- 6.3 TB of scatter traffic at 100^3 for 4 % of the flops --
// and runs 909 dependent levels.
//
// The plan therefore factors a COARSER partition of the same matrix: chains
// s, s+1, ..., e of consecutive supernodes with
//   * parent(s) = s+1 (the first block row below the diagonal of L(:,s)),
//   * symmetric structure (U(s,:)'s columns = L(:,s)'s rows below the
//     diagonal block),
//   * nested structure: the rows of L(:,s) below s lie in s+1 or below s+1,
//   * total width <= 256 and at most ZERO_FRAC of the merged storage being
//     explicit zeros
// become one supernode J whose L block column holds cols(J) u below(e) (in
// e's row order) and whose U block row holds segments [first member row
// holding the column, end of J).  The union of the members' structures is
// the structure of e's update, so every Schur update of the coarse partition
// lands on stored positions, and a structural zero stays an exact zero (all
// of its products have a zero factor): the factors are the reference's, with
// the order of additions changed.
//
// The coarse LUstruct is described in the reference formats (so the
// ordinary plan runs it) and values move between the two layouts by the
// expand / compress programs below: per original L block column one
// descriptor plus one merged row position per stored row; per original U
// block one descriptor, one first-row per column and a per-(merged row,
// column) base table D, so that a U segment (a, g) lands at D + fst.
#pragma once
#include <cstdint>
#include <vector>

#include "slu_abi.h"

namespace slu {

struct Amalg {
    int64_t n = 0;
    int ns1 = 0, ns2 = 0;            // original / merged supernodes
    std::vector<int_t> xsup2;        // ns2 + 1
    std::vector<int_t> supno2;       // n
    std::vector<int> grp;            // original supernode -> merged
    // merged LUstruct, 1x1, flat reference formats (slu_lustruct_build's inputs)
    std::vector<int_t> Lidx2, Uidx2;
    std::vector<int64_t> Loff2, Lvoff2, Uoff2, Uvoff2; // per merged supernode, -1 if empty
    int64_t lval2 = 0, uval2 = 0;                       // value counts (no spare element)
    // original value layout: contiguous per block column / row in supernode order
    int64_t lval1 = 0, uval1 = 0;

    // ---- expand / compress programs
    struct LCol {        // one original L block column
        int64_t src;     // value offset in the original L values
        int64_t dst;     // merged value offset of its first column
        int64_t map;     // offset of its row positions in lrow
        int32_t nsupr;   // original rows
        int32_t w;       // columns
        int32_t ld2;     // merged leading dimension
        int32_t pad;
    };
    struct URowX {       // one original U block row a
        int64_t src;     // value offset of its first segment in the original U values
        int64_t c0;      // first of its column entries in ucol
        int32_t nc;      // column entries (all columns of all its blocks)
        int32_t end;     // xsup[a + 1]
        int32_t w;       // width of a (segments are at most this long)
        int32_t pad;
    };
    std::vector<LCol> lcols;
    std::vector<int32_t> lrow;  // merged row position of every stored original L row
    std::vector<URowX> urows;
    // per original U column entry (block order, column order): the D index
    // of its coarse destination (>= DL0: inside the coarse diagonal block, in
    // the coarse L) and the first row of its segment
    std::vector<int32_t> ucol;  // interleaved (didx, fst)
    int64_t DL0 = 0;
    std::vector<int64_t> D;     // merged destination base per (merged row, column)
    int64_t n_merged_groups = 0, zeros = 0;
    bool programs = true; // false: the coarse structure only (no expand / compress programs)
    // algorithmic work of the ORIGINAL partition (the reference's accounting,
    // SURVEY 8d; the plan's own counts are the coarse partition's): real-flop
    // sums, weighted by value type in the plan
    double fl_schur = 0;          // sum over U columns of 2 * m * seglen
    double fl_trsm = 0;           // sum w (w + 1) m
    double fl_trsv = 0;           // sum seglen (seglen + 1)
    double fl_s1 = 0, fl_s2 = 0, fl_w = 0; // diagonal LU: w(w-1)/2, (w-1)w(2w-1)/6, w

    // Builds everything from a 1x1 LUstruct's index arrays.  Returns false
    // when no two supernodes merge (the plan then runs the original).
    bool build(int64_t n, int nsupers, const int_t *xsup, const int_t *const *lidx,
               const int_t *const *uidx, double zero_frac, int maxw);

    // The coarse partition as a symbolic factorization (symbfact's
    // Glu_freeable arrays, for the structural distribute on any grid):
    // lsub of supernode J at xlsub[first column of J], U segment starts per
    // column in xusub / usub.
    void coarse_glu(std::vector<int_t> &xlsub, std::vector<int_t> &lsub,
                    std::vector<int_t> &xusub, std::vector<int_t> &usub) const;

    // Host versions of the device programs (tests): dir 0 expands the
    // original values into zeroed merged arrays, dir 1 compresses back.
    template <typename T> void apply(T *oL, T *oU, T *mL, T *mU, int dir) const;
};

} // namespace slu
