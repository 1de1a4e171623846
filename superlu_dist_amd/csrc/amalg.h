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
#include <functional>
#include <vector>

#include "common.h"
#include "slu_abi.h"

namespace slu {

// The original partition's algorithmic work (the reference's accounting,
// SURVEY 8d): real-flop sums, weighted by value type in the plan.
struct AmalgFlops {
    double schur = 0; // sum over U columns of 2 * m * seglen
    double trsm = 0;  // sum w (w + 1) m
    double trsv = 0;  // sum seglen (seglen + 1)
    double s1 = 0, s2 = 0, w = 0; // diagonal LU: w(w-1)/2, (w-1)w(2w-1)/6, w
};

// Passes 1 + 2 of the analysis over the supernodes [a0, a1): per-supernode
// structure facts (parent, symmetric, nested) and the greedy chains, which
// never cross a1.  lidx / uidx (1x1 reference format, every block of the
// supernode) need to be valid for [a0, a1) only.  Returns the first
// supernode of every group in the range; fl (if given) gets the range's
// original-partition work added; ucne (if given) the non-empty U column
// entries of every supernode of the range.
std::vector<int> amalg_chains(int64_t n, int ns, const int_t *xsup, const int_t *const *lidx,
                              const int_t *const *uidx, double zero_frac, int maxw, int a0, int a1,
                              AmalgFlops *fl, std::vector<int64_t> *ucne = nullptr);

// Relayout programs (device kernels in amalg_dev.h, host mirrors in the
// apply functions).  A column range [c0, c1) of one L block column whose
// rows go through a row map: k_amalg_l dir 0: m[dst + c ld2 + lrow[map + i]]
// = o[src + c nsupr + i]; dir 1 the reverse.
struct LColX {
    int64_t src, dst, map;
    int32_t nsupr, c0, c1, ld2;
};
// <= 64 non-empty column segments of one U block row: segment j is
// o[src + ...] (segments back to back), rows [end - len, end) with len =
// ucl[c0 + j] + 1, landing at D[ucd[c0 + j]] + end - len in the coarse L
// (index >= DL0) or U values.  Empty segments (the reference stores a first
// row = end for them) have no program entry: 6 bytes per non-empty column
// (100^3: 129 M of the 310 M column entries are non-empty; lengths <= the
// widest supernode, 512).
struct UChunk {
    int64_t src; // value offset of the chunk's first segment (caller's layout)
    int64_t c0;  // first column entry in ucd / ucl
    int32_t nc;  // <= 64
    int32_t end; // xsup[a + 1] of the row
};
// a contiguous range copy to[dst + i] = from[src + i], i < len (k_ranges)
struct GaSpan {
    int64_t src, dst;
    int64_t len;
};

struct Amalg {
    int64_t n = 0;
    int ns1 = 0, ns2 = 0;            // original / merged supernodes
    std::vector<int_t> xsup2;        // ns2 + 1
    std::vector<int_t> supno2;       // n
    std::vector<int> grp;            // original supernode -> merged
    // merged LUstruct, 1x1, flat reference formats (slu_lustruct_build's inputs)
    RawVec<int_t> Lidx2, Uidx2;      // (every entry written by the analysis)
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
        int64_t c0;      // first of its non-empty column entries in ucd / ucl
        int32_t nc;      // non-empty column entries (over all its blocks)
        int32_t end;     // xsup[a + 1]
        int32_t w;       // width of a (segments are at most this long)
        int32_t pad;
    };
    std::vector<LCol> lcols;
    RawVec<int32_t> lrow;       // merged row position of every stored original L row
    std::vector<URowX> urows;
    // per non-empty original U column entry (block order, column order): the
    // D index of its coarse destination (>= DL0: inside the coarse diagonal
    // block, in the coarse L) and its segment length - 1
    RawVec<int32_t> ucd;
    RawVec<uint16_t> ucl;
    int64_t DL0 = 0;
    RawVec<int64_t> D;          // merged destination base per (merged row, column)
    int64_t n_merged_groups = 0, zeros = 0;
    bool programs = true; // false: the coarse structure only (no expand / compress programs)
    // called by build() once lval2 / uval2 are known (before the coarse
    // index arrays and the programs are built): the plan allocates the coarse
    // storage beside the rest of the analysis
    std::function<void(int64_t, int64_t)> on_sizes;
    // algorithmic work of the ORIGINAL partition (the reference's accounting,
    // SURVEY 8d; the plan's own counts are the coarse partition's): real-flop
    // sums, weighted by value type in the plan
    double fl_schur = 0;          // sum over U columns of 2 * m * seglen
    double fl_trsm = 0;           // sum w (w + 1) m
    double fl_trsv = 0;           // sum seglen (seglen + 1)
    double fl_s1 = 0, fl_s2 = 0, fl_w = 0; // diagonal LU: w(w-1)/2, (w-1)w(2w-1)/6, w

    // Builds everything from a 1x1 LUstruct's index arrays.  Returns false
    // when no two supernodes merge (the plan then runs the original).  With
    // defer_programs, build() stops after the coarse index arrays and
    // build_programs() (which needs the same index arrays alive) builds D and
    // the expand / compress programs: the plan runs it beside the coarse plan.
    bool build(int64_t n, int nsupers, const int_t *xsup, const int_t *const *lidx,
               const int_t *const *uidx, double zero_frac, int maxw);
    bool defer_programs = false;
    void build_programs();
    // the LUstruct's index arrays for a deferred build_programs(): the
    // pointer tables build() was given need not outlive it
    void set_index(const int_t *const *lidx, const int_t *const *uidx);
    Amalg();
    ~Amalg();
    Amalg(const Amalg &) = delete;
    Amalg &operator=(const Amalg &) = delete;
    struct URow;
    struct Work;
    std::unique_ptr<Work> work;

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

// ------------------------------------------------------------------ grids
// Amalgamation of a caller's LUstruct on a Pr x Pc grid (the block-cyclic
// layout of SRC/pddistribute.c: block (I, J) on rank (I mod Pr, J mod Pc)).
// No rank holds the whole structure, and a coarse block (grp(I), grp(J))
// lives on another rank than most of its fine blocks, so:
//   1. every rank sends the structure of its blocks to the ANALYSIS OWNER of
//      their supernode (contiguous supernode ranges, one per rank), which
//      rebuilds the 1x1 index arrays of its range and runs passes 1 + 2 of
//      the analysis (amalg_chains; chains never cross a range end);
//   2. the ranges' group starts are all-gathered: every rank knows grp;
//   3. every fine block goes to the owner of its coarse block -- its
//      structure once at plan time (the receiver builds its local coarse
//      LUstruct, the union of what arrives, and the unpack programs), its
//      values at every upload (pack -> all-to-all -> unpack) and back at
//      download (the reverse).
// The phases are pure functions of their inputs, so the CPU tests run all
// ranks of a grid in one process (ga_simulate) and the engine runs one rank
// with the transport's all-to-all between them.
struct GaFine { // one rank's view of the caller's (fine) LUstruct
    int64_t n = 0;
    int ns = 0, Pr = 1, Pc = 1, myrow = 0, mycol = 0;
    const int_t *xsup = nullptr;
    const int_t *const *lidx = nullptr; // nlc local block columns (reference format) or null
    const int_t *const *uidx = nullptr; // nlr local block rows
    int nlc() const { return (ns + Pc - 1) / Pc; }
    int nlr() const { return (ns + Pr - 1) / Pr; }
    int P() const { return Pr * Pc; }
    int iam() const { return myrow * Pc + mycol; }
};
using GaStreams = std::vector<std::vector<int64_t>>; // one per peer rank

// supernodes [ga_range(ns, P, r), ga_range(ns, P, r + 1)) are rank r's to analyse
inline int ga_range(int ns, int P, int r) { return (int)((int64_t)ns * r / P); }
int ga_owner(int ns, int P, int s);

// phase 1: the structure of my blocks, per analysis owner
GaStreams ga_structure_out(const GaFine &f);
// phase 1 (owner): chains of my range from every rank's stream
struct GaChains {
    std::vector<int64_t> gstart; // first supernode of every group of my range
    AmalgFlops fl;               // my range's original-partition work
};
GaChains ga_analyse(const GaFine &f, const GaStreams &in, double zero_frac, int maxw);
// phase 2: the partition from every range's group starts (rank order)
struct GaPartition {
    int ns2 = 0;
    std::vector<int> grp;        // fine supernode -> coarse
    std::vector<int_t> xsup2, supno2;
};
GaPartition ga_partition(const GaFine &f, const std::vector<std::vector<int64_t>> &gstarts);
// phase 3: one rank's relayout
struct GaRelay {
    // ---- send side (pack programs read the caller's local values)
    GaStreams sstruct;           // per destination: structure of its pieces
    std::vector<int64_t> scount; // per destination: values
    std::vector<int64_t> soff;   // per destination: first value in the send buffer (P + 1)
    std::vector<int64_t> lsrc, usrc; // caller value offset per local block column / row
    int64_t lval = 0, uval = 0;      // caller local value counts
    std::vector<LColX> pack_l;       // o = send buffer, m = caller L (k_amalg_l, dir 1)
    std::vector<int32_t> pack_lrow;  // caller local row of every packed L row
    std::vector<GaSpan> pack_u;      // caller U -> send buffer
    // ---- receive side
    std::vector<int64_t> rcount, roff; // per source: values, first value in the receive buffer
    int nlc2 = 0, nlr2 = 0;
    std::vector<std::vector<int_t>> Lidx2, Uidx2; // local coarse block columns / rows (empty: none)
    std::vector<int64_t> Lvoff2, Uvoff2;          // -1 where empty
    int64_t lval2 = 0, uval2 = 0;
    std::vector<LColX> unpack_l;      // o = receive buffer, m = coarse L (k_amalg_l, dir 0)
    std::vector<int32_t> unpack_lrow; // coarse local row of every received L row
    std::vector<UChunk> unpack_u;     // o = receive buffer (k_amalg_u, dir 0)
    std::vector<int32_t> unpack_ucd;  // D index per received non-empty U column
    std::vector<uint16_t> unpack_ucl; // its segment length - 1
    std::vector<int64_t> D;
    int64_t DL0 = 0;
    int64_t received = 0; // values in the receive buffer
};
void ga_send_side(const GaFine &f, const GaPartition &g, GaRelay &r);
void ga_receive_side(const GaFine &f, const GaPartition &g, const GaStreams &in, GaRelay &r);

// Host mirrors of the device programs (tests).  pack: caller L / U -> send
// buffer; unpack: receive buffer -> coarse (zeroed by the caller); dir 1
// of each runs the reverse copy.
template <typename T> void ga_pack(const GaRelay &r, T *cL, T *cU, T *send, int dir);
template <typename T> void ga_unpack(const GaRelay &r, T *recv, T *mL, T *mU, int dir);

} // namespace slu
