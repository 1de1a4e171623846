/*
 * slu_mi355x.h -- C ABI of libslu_mi355x.so, the MI355X-native numeric
 * factorization engine for SuperLU_DIST.
 *
 * Three groups of entry points:
 *
 * 1. Drop-in replacements (identical prototypes to the reference):
 *      pdgstrf  -- SRC/superlu_ddefs.h:530-531, implemented at SRC/pdgstrf.c:242
 *      psgstrf  -- SRC/superlu_sdefs.h:507,     implemented at SRC/psgstrf.c
 *      pzgstrf  -- SRC/superlu_zdefs.h:507,     implemented at SRC/pzgstrf.c
 *      dscatter_l / dscatter_u   SRC/superlu_ddefs.h:519-528 (+ s/z),
 *      dscatter_l_1              SRC/dscatter.c:29-43 (no header prototype; its
 *                                usub / lsub are int *, not int_t *),
 *        exported because the reference's pdgstrf.c.o defines them
 *        (SRC/pdgstrf.c:171 #includes SRC/dscatter.c) and dscatter3d.c.o
 *        still references them after pdgstrf.c.o is removed.
 *      sp_colorder -- SRC/superlu_defs.h:1079, implemented at SRC/sp_colorder.c:81
 *      symbfact    -- SRC/superlu_defs.h:1091, implemented at SRC/symbfact.c:81
 *        (the column ordering post-pass and symbolic factorization pdgssvx
 *        runs before pddistribute; declared with group 3 below)
 *    On multi-rank grids pdgstrf uses the MPI communicators in gridinfo_t to
 *    bootstrap RCCL (or, when ranks share a GPU, to carry the host-staged
 *    panel broadcasts) and for the final info reduction; the MPI symbols are
 *    resolved from the host process at run time, so this library has no
 *    link-time MPI dependency.
 *
 * 2. Engine API (no MPI): the same factorization driven by a caller that
 *    bootstraps RCCL itself (bench.py / tests through torch.distributed).
 *
 * 3. Front-end helpers used by tests and the benchmark to build LUstructs for
 *    stencil matrices (geometric nested dissection, supernodal symbolic
 *    factorization, 2D block-cyclic distribution in the reference layout of
 *    SRC/pddistribute.c:327-2400).
 *
 * All functions are extern "C"; no C++ exception crosses this boundary.
 */
#ifndef SLU_MI355X_H
#define SLU_MI355X_H

#include "slu_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- 1. drop-in entry points ---------------- */
int_t pdgstrf(superlu_dist_options_t *options, int m, int n, double anorm,
              dLUstruct_t *LUstruct, gridinfo_t *grid, SuperLUStat_t *stat,
              int *info);
int_t psgstrf(superlu_dist_options_t *options, int m, int n, float anorm,
              sLUstruct_t *LUstruct, gridinfo_t *grid, SuperLUStat_t *stat,
              int *info);
int_t pzgstrf(superlu_dist_options_t *options, int m, int n, double anorm,
              zLUstruct_t *LUstruct, gridinfo_t *grid, SuperLUStat_t *stat,
              int *info);

void dscatter_l_1(int ib, int ljb, int nsupc, int_t iukp, int_t *xsup,
                  int klst, int nbrow, int_t lptr, int temp_nbrow,
                  int *usub, int *lsub, double *tempv,
                  int *indirect_thread, int_t **Lrowind_bc_ptr,
                  double **Lnzval_bc_ptr, gridinfo_t *grid);
void dscatter_l(int ib, int ljb, int nsupc, int_t iukp, int_t *xsup,
                int klst, int nbrow, int_t lptr, int temp_nbrow,
                int_t *usub, int_t *lsub, double *tempv,
                int *indirect_thread, int *indirect2,
                int_t **Lrowind_bc_ptr, double **Lnzval_bc_ptr,
                gridinfo_t *grid);
void dscatter_u(int ib, int jb, int nsupc, int_t iukp, int_t *xsup,
                int klst, int nbrow, int_t lptr, int temp_nbrow,
                int_t *lsub, int_t *usub, double *tempv,
                int_t **Ufstnz_br_ptr, double **Unzval_br_ptr,
                gridinfo_t *grid);
void sscatter_l_1(int ib, int ljb, int nsupc, int_t iukp, int_t *xsup,
                  int klst, int nbrow, int_t lptr, int temp_nbrow,
                  int *usub, int *lsub, float *tempv,
                  int *indirect_thread, int_t **Lrowind_bc_ptr,
                  float **Lnzval_bc_ptr, gridinfo_t *grid);
void sscatter_l(int ib, int ljb, int nsupc, int_t iukp, int_t *xsup,
                int klst, int nbrow, int_t lptr, int temp_nbrow,
                int_t *usub, int_t *lsub, float *tempv,
                int *indirect_thread, int *indirect2,
                int_t **Lrowind_bc_ptr, float **Lnzval_bc_ptr,
                gridinfo_t *grid);
void sscatter_u(int ib, int jb, int nsupc, int_t iukp, int_t *xsup,
                int klst, int nbrow, int_t lptr, int temp_nbrow,
                int_t *lsub, int_t *usub, float *tempv,
                int_t **Ufstnz_br_ptr, float **Unzval_br_ptr,
                gridinfo_t *grid);
void zscatter_l_1(int ib, int ljb, int nsupc, int_t iukp, int_t *xsup,
                  int klst, int nbrow, int_t lptr, int temp_nbrow,
                  int *usub, int *lsub, doublecomplex *tempv,
                  int *indirect_thread, int_t **Lrowind_bc_ptr,
                  doublecomplex **Lnzval_bc_ptr, gridinfo_t *grid);
void zscatter_l(int ib, int ljb, int nsupc, int_t iukp, int_t *xsup,
                int klst, int nbrow, int_t lptr, int temp_nbrow,
                int_t *usub, int_t *lsub, doublecomplex *tempv,
                int *indirect_thread, int *indirect2,
                int_t **Lrowind_bc_ptr, doublecomplex **Lnzval_bc_ptr,
                gridinfo_t *grid);
void zscatter_u(int ib, int jb, int nsupc, int_t iukp, int_t *xsup,
                int klst, int nbrow, int_t lptr, int temp_nbrow,
                int_t *lsub, int_t *usub, doublecomplex *tempv,
                int_t **Ufstnz_br_ptr, doublecomplex **Unzval_br_ptr,
                gridinfo_t *grid);

/* ---------------- 2. engine API ---------------- */

/* value type codes */
enum { SLU_D = 0, SLU_S = 1, SLU_Z = 2 };

/* One communicator context per 2D grid: RCCL world/row/column communicators
 * plus the device this rank drives.  uid is an ncclUniqueId (128 bytes)
 * created by slu_comm_unique_id on world rank 0 and broadcast by the caller.
 * For a 1x1 grid pass uid = NULL (no RCCL is created). */
typedef struct slu_comm slu_comm;
int slu_comm_unique_id(void *uid_out128);
slu_comm *slu_comm_create(const void *uid128, int nprow, int npcol, int iam,
                          int device);
/* Test transport: broadcasts are staged through host memory and delegated
 * to fn (group 0 = whole grid, 1 = my process row, 2 = my process column;
 * root = rank within that group; buf holds bytes bytes, valid on the root
 * and to be filled on the others).  Lets several ranks share one GPU, which
 * RCCL refuses ("Duplicate GPU"); the kernels are the same as with RCCL. */
typedef int (*slu_host_bcast_fn)(void *ctx, int group, int root, void *buf,
                                 int64_t bytes);
slu_comm *slu_comm_create_host(slu_host_bcast_fn fn, void *ctx, int nprow,
                               int npcol, int iam, int device);
/* Point-to-point test transport: every exchange phase hands fn the list of
 * sends and receives (peer = rank within group, as ncclSend / ncclRecv get
 * it) that the RCCL transport issues inside one ncclGroupStart / End, in the
 * same order, with host-staged buffers; fn must post all of them before
 * waiting for any (e.g. torch.distributed isend / irecv + wait) and return 0
 * once all completed.  Sends and receives between one pair of ranks match in
 * order, as in RCCL.  device = -1: no GPU (schedule-only plans). */
typedef struct {
    int group;     /* 0 whole grid, 1 my process row, 2 my process column */
    int peer;      /* rank within that group */
    int send;      /* 1 send, 0 receive */
    int reserved;
    void *buf;
    int64_t bytes;
} slu_host_p2p_op;
typedef int (*slu_host_p2p_fn)(void *ctx, int nops, const slu_host_p2p_op *ops);
slu_comm *slu_comm_create_host_p2p(slu_host_p2p_fn fn, void *ctx, int nprow,
                                   int npcol, int iam, int device);
/* 3D grids (the reference's gridinfo3d_t, SRC/superlu_grid3d.c; pdgstrf3d,
 * SRC/pdgstrf3d.c:121): npdep (a power of two) layers of an nprow x npcol
 * grid, rank iam3d = layer * nprow * npcol + row * npcol + column.  Group 3
 * of the communicator joins the ranks at my (row, column) of every layer
 * (the reference's grid3d->zscp); the plan of a 3D communicator factors the
 * layer's forests of the supernodal etree and reduces the ancestors between
 * layers (see slu_plan_gather3d).  The _host_p2p3d variant is the
 * point-to-point test transport with group 3 added (peer = layer). */
slu_comm *slu_comm_create3d(const void *uid128, int nprow, int npcol, int npdep,
                            int iam3d, int device);
slu_comm *slu_comm_create_host_p2p3d(slu_host_p2p_fn fn, void *ctx, int nprow,
                                     int npcol, int npdep, int iam3d, int device);
/* Ranks in group 0 / 1 / 2 / 3 of c (for RCCL: ncclCommCount of the layer's
 * world / row / column communicator or of the layer group), -1 on error. */
int slu_comm_size(const slu_comm *c, int group);
void slu_comm_destroy(slu_comm *c);

/* Engine options (everything the kernels need beyond the LUstruct). */
typedef struct {
    int replace_tiny_pivot; /* options->ReplaceTinyPivot */
    int timing;             /* 1: per-phase HIP events; 2: + per-level log on stderr */
    int serial;             /* 1: one stream, no look-ahead overlap (kernel profiling) */
    int overlap_upload;     /* 1: slu_plan_create starts the H2D copy of the L/U
                               values as soon as their HBM is allocated and
                               builds the rest of the plan meanwhile;
                               slu_plan_upload then waits for it */
    int overlap_download;   /* 1: slu_plan_factor copies each finished level's
                               L columns / U rows back into the host LUstruct
                               while later levels are factored (the
                               factors are final once their level's panels
                               are done); slu_plan_download is then a no-op */
    int schedule_only;      /* 1: host-only plan (no HIP call at all): layout,
                               index exchange, levels and exchange sections,
                               for slu_plan_check_exchange; a grid needs the
                               point-to-point host transport */
    const int64_t *forest_map; /* 3D grids: per supernode its forest in heap
                               order (0 = top ancestors), e.g. the reference's
                               dtrf3Dpartition_t.supernode2treeMap; NULL: the
                               engine's own partition (SRC/supernodalForest.c) */
} slu_engine_opts;

/* A plan = device-resident factors + every index table the kernels use.
 * Built from a host LUstruct (any of d/s/z by dtype), once per structure. */
typedef struct slu_plan slu_plan;
slu_plan *slu_plan_create(int dtype, void *LUstruct, int n, int nprow,
                          int npcol, int iam, slu_comm *comm,
                          const slu_engine_opts *opts, char *err, int errlen);
/* (Re)load the numeric values of the host LUstruct into HBM. */
int slu_plan_upload(slu_plan *p);
/* Numeric factorization on the device (inputs resident in HBM).
 * anorm is used for the tiny-pivot threshold as in SRC/pdgstrf.c:412-413. */
int slu_plan_factor(slu_plan *p, double anorm, int *info, int *tiny_pivots);
/* Upload the host LUstruct's values as FINISHED factors (e.g. from an
 * earlier pdgstrf): the device storage then serves slu_plan_solve / refine
 * without a factorization. */
int slu_plan_adopt_factors(slu_plan *p);
/* Keep a pristine device copy of the uploaded values (snapshot) and restore
 * the working factor storage from it (benchmark repetitions; device-to-device). */
int slu_plan_snapshot(slu_plan *p);
int slu_plan_restore(slu_plan *p);
/* Change the measurement options of an existing plan (timing, serial). */
int slu_plan_set_timing(slu_plan *p, int timing, int serial);
/* Wait for all work of the plan's stream. */
int slu_plan_sync(slu_plan *p);
/* Copy factors back into the host LUstruct arrays. */
int slu_plan_download(slu_plan *p);
/* Solve L U x = b with the device-resident factors of the last
 * slu_plan_factor (the supernodal solve of SRC/pdgstrs.c
 * in the LUstruct's permuted coordinates).  b: host array of nrhs columns of
 * n values (ld ldb, element type of the plan), overwritten with x.  On a 2D
 * grid the call is collective: every rank passes the same b and gets the
 * whole x; partial sums of a block row are reduced along its process row to
 * the diagonal owner and solved pieces travel down the owner's process
 * column (pdgstrs_lsum.c's scheme, level by level).  t_solve_ms in the stats
 * is the device time of the last call. */
int slu_plan_solve(slu_plan *p, void *b, int64_t ldb, int nrhs);
/* Device-side refill of the factor storage from new values of A with the
 * same pattern (replaces the options->Fact ==
 * SamePattern_SameRowPerm branch of pddistribute, SRC/pddistribute.c:545-672).
 * set_a_pattern: A in the LUstruct's permuted coordinates (what
 * dReDistribute_A hands pddistribute, SRC/pddistribute.c:536), CSC with
 * column pointers xa[ncol+1] and row indices asub[xa[ncol]]; entries of
 * other process rows / columns are ignored, so every rank may pass the
 * whole matrix.  Fails (-1) if an entry lies outside the L/U structure.
 * fill_a: zero this rank's L and U values and store a[e] (nnz values of the
 * plan's element type, host pointer or, with on_device = 1, device pointer)
 * at their positions; a duplicated (row, column) keeps the last value.
 * t_fill_ms in the stats is the device time of the zero + scatter. */
int slu_plan_set_a_pattern(slu_plan *p, int64_t ncol, const int64_t *xa, const int64_t *asub);
int slu_plan_fill_a(slu_plan *p, const void *a, int on_device);
/* Iterative refinement on the device (SRC/pdgsrfs.c:197-253, the LUstruct's
 * permuted coordinates; on a 2D grid collective, b and x replicated, the
 * residual as pdgsmv's: each rank's entries of A give partial rows, reduced
 * along process rows to the diagonal owners): for each of the nrhs columns of b / x
 * (ld ld, host arrays of the plan's element type), repeat R = b - A x,
 * berr = max_i |R_i| / (|A||x| + |b|)_i (SAFE1/SAFE2 guards), and while
 * berr > eps, berr <= lstres / 2 and fewer than 20 steps, x += solve(R) with
 * the device factors.  A = the values of the last slu_plan_fill_a (a device
 * pointer passed there must stay valid).  x: in = initial solution (e.g.
 * from slu_plan_solve), out = refined.  berr[nrhs], steps[nrhs] (may be
 * NULL) receive the final backward error and the number of steps
 * (stat->RefineSteps).  t_refine_ms in the stats = device time of the call. */
int slu_plan_refine(slu_plan *p, const void *b, void *x, int64_t ld, int nrhs, double *berr,
                    int *steps);
/* Schedule-only plans: replay every level's exchange phases of
 * slu_plan_factor through the communicator on host buffers; each received
 * section is checked byte for byte against what its root wrote.  Collective;
 * returns 0 and the number / bytes of sections this rank received. */
int slu_plan_check_exchange(slu_plan *p, int64_t *nsections, int64_t *nbytes);
/* 3D plans, after slu_plan_factor (collective over the layers): the factored
 * forests travel to layer 0, whose ranks then hold every supernode's final
 * L / U values (pdgssvx3d's dgatherAllFactoredLU, SRC/pd3dcomm.c:816);
 * the other layers' storage is left partial.  slu_plan_download then gives
 * the factors on layer 0. */
int slu_plan_gather3d(slu_plan *p);
void slu_plan_destroy(slu_plan *p);

/* Plan statistics (algorithmic work of one factorization on this rank). */
typedef struct {
    int64_t nsupers, nlevels;
    int64_t n_schur_tiles, n_diag, n_trsm_items;
    double schur_flops;        /* exact, unpadded: sum 2*nrows*seglen */
    double schur_flops_padded; /* reference accounting 2*m*ncols*ldu */
    double panel_flops;        /* diag LU + TRSM + TRSV (SRC/pdgstrf2.c) */
    double scatter_bytes;      /* 3*sizeof(T)*m*ncols summed */
    double lu_bytes;           /* device bytes of L and U values */
    double index_bytes;        /* device bytes of plan index tables */
    /* timing of the last slu_plan_factor (ms), when opts.timing */
    double t_total_ms, t_diag_ms, t_trsm_ms, t_schur_ms, t_comm_ms;
    double t_schur_big_ms;     /* k_schur_big launches (128x128 tiles) */
    double schur_big_flops;    /* flops of the supernodes on 128x128 tiles */
    int64_t n_schur_launches;
    int64_t n_schur_big_launches;
    double comm_bytes;         /* bytes of the broadcast sections this rank
                                  takes part in (as root or receiver) per factor */
    double t_solve_ms;         /* device time of the last slu_plan_solve */
    double t_fill_ms;          /* device time of the last slu_plan_fill_a */
    double t_refine_ms;        /* device time of the last slu_plan_refine */
    /* host wall times of the drop-in path (ms) */
    double t_plan_ms;          /* slu_plan_create */
    double t_upload_ms;        /* H2D of the L/U values (overlapped with the
                                  plan build when opts.overlap_upload) */
    double t_upload_wait_ms;   /* of which slu_plan_upload still waited */
    double t_d2h_ms;           /* D2H of the factors (overlap_download: the
                                  helper thread's whole span) */
    double t_d2h_tail_ms;      /* D2H after the device finished the factorization */
    double h2d_bytes, d2h_bytes;
    int64_t n_d2h_copies;
    double comm_buf_bytes;     /* HBM of the receive ring (diag packages + panels) */
    /* engine-side amalgamation (csrc/amalg.h, 1x1 grids): nsupers above is
     * the factored (coarse) partition, nsupers_in the caller's */
    int64_t nsupers_in;
    int64_t amalg_groups;      /* merged supernodes of more than one original */
    double amalg_zeros;        /* explicit zeros the coarse storage adds */
    double t_amalg_ms;         /* host analysis + programs (part of t_plan_ms) */
    double t_expand_ms;        /* device relayout caller -> coarse (last upload) */
    double t_compress_ms;      /* device relayout coarse -> caller (last download) */
    /* 3D grids (timing on): device time of each of this layer's phases
     * (phase p = the forest at level p, 0 = leaves) and of its ancestor
     * reductions, last slu_plan_factor */
    double t_phase_ms[8];
    double t_zreduce_ms;
    double zred_bytes[8];      /* 3D: bytes of the reduction after each phase */
    int64_t npdep, zlayer, phase_last; /* 3D: layers, mine, my last phase */
} slu_plan_stats;
int slu_plan_get_stats(const slu_plan *p, slu_plan_stats *st);

/* Last error string of this thread (empty when none). */
const char *slu_last_error(void);
/* Test hook: fill the LDS of every CU of `device` with NaN, so that a
 * kernel reading LDS it did not write fails deterministically. */
int slu_debug_poison_lds(int device);

/* ---------------- 3. front-end helpers ---------------- */

/* Sparse matrix in compressed-column form, values of the given dtype
 * (complex = interleaved re,im doubles). */
typedef struct {
    int64_t n, nnz;
    int64_t *colptr; /* n+1 */
    int64_t *rowind; /* nnz */
    void *val;       /* nnz values */
    int dtype;
} slu_csc;

/* kind: 0 = 2D 5-point, 1 = 3D 7-point, 2 = 3D 27-point.
 * Row r = (i*ny + j)*nz + l (lexicographic), diagonal diag (+ i*diag_im for
 * complex), every off-diagonal neighbour = off. */
slu_csc *slu_gen_stencil(int kind, int nx, int ny, int nz, double diag,
                         double diag_im, double off, int dtype);
slu_csc *slu_csc_create(int64_t n, int64_t nnz, const int64_t *colptr,
                        const int64_t *rowind, const void *val, int dtype);
void slu_csc_free(slu_csc *A);

/* Geometric nested dissection of an nx*ny*nz grid (nz=1 for 2D).
 * perm_c[i] = position of column i in the new order (SuperLU convention). */
int slu_order_nd_grid(int nx, int ny, int nz, int64_t *perm_c);

/* Symbolic factorization of P(A+A^T)P^T (structure of the LU factors when A
 * is structurally symmetric; a valid superset otherwise).  perm_c is
 * composed with an etree postorder.  relax / maxsup as sp_ienv_dist(2/3).
 * flags: SLU_SYMB_MULTICHILD lets a chain supernode continue through a
 * column with several etree children (shorter supernodal trees for
 * level-set nested dissections).  SLU_SYMB_REFERENCE instead runs pdgssvx's
 * own symbolic stage (sp_colorder + symbfact below, SRC/pdgssvx.c:1046-1076,
 * perm_r = I): supernodes and structure are the reference's, and
 * slu_distribute then lays them out with the reference's pddistribute
 * (slu_distribute_glu on Pc A Pc^T).  SLU_SYMB_REFERENCE | SLU_SYMB_COARSE
 * then replaces the partition by the engine's coarse one (the amalgamation a
 * 1x1 plan applies internally, csrc/amalg.h), so that it can be distributed
 * on any grid; slu_symb_ref_info keeps the reference partition's size and
 * work. */
enum { SLU_SYMB_MULTICHILD = 1, SLU_SYMB_REFERENCE = 2, SLU_SYMB_COARSE = 4 };
typedef struct slu_symb slu_symb;
slu_symb *slu_symbolic(const slu_csc *A, const int64_t *perm_c, int relax,
                       int maxsup, int flags);
void slu_symb_free(slu_symb *s);
int64_t slu_symb_nsupers(const slu_symb *s);
/* copies: xsup (nsupers+1), supno (n), final perm_c (n) */
void slu_symb_arrays(const slu_symb *s, int64_t *xsup, int64_t *supno,
                     int64_t *perm_c);
/* nnz(L) including the diagonal blocks, nnz(U) excluding them */
void slu_symb_counts(const slu_symb *s, double *nnzL, double *nnzU);
/* SLU_SYMB_REFERENCE: [nsupers of the reference's partition, schur, trsm,
 * trsv, s1, s2, w] -- the algorithmic-work sums of that partition (real
 * flops; the plan's weights per value type, csrc/amalg.h) */
void slu_symb_ref_info(const slu_symb *s, double *out);
/* |struct(L_s)| (rows incl. the diagonal block) per supernode */
void slu_symb_struct_sizes(const slu_symb *s, int64_t *sizes);

/* ---- Column ordering post-pass + symbolic factorization,
 * the reference's arrays bit for bit (csrc/symbolic.cpp, tests/test_symbolic.py).
 *
 * slu_colorder replaces sp_colorder (SRC/sp_colorder.c:81): colbeg / colend
 * (n each) get A Pc''s column pointers; with recompute (Fact = DOFACT or
 * SamePattern) etree (n) gets the etree of Pc(A'+A)Pc' (ata != 0 or m != n:
 * the column etree of A Pc'), postordered, and perm_c follows the postorder.
 * Returns 0, or -1 (slu_last_error). */
int slu_colorder(int64_t m, int64_t n, const int64_t *colptr, const int64_t *rowind, int ata,
                 int recompute, int64_t *perm_c, int64_t *etree, int64_t *colbeg,
                 int64_t *colend);
/* slu_symbfact replaces symbfact (SRC/symbfact.c:81) on A Pc' (colbeg / colend
 * from slu_colorder, rowind relabelled by perm_c as SRC/pdgssvx.c:1053-1058
 * does) with the postordered etree.  NULL on a structurally zero diagonal
 * (the reference ABORTs).  sizes: [nsupers, |lsub|, |usub|, nnzL, nnzU,
 * nnzLU, lsub size before compression (symbfact returns its negative)]. */
void *slu_symbfact(int64_t m, int64_t n, const int64_t *colbeg, const int64_t *colend,
                   const int64_t *rowind, const int64_t *etree, int64_t relax,
                   int64_t maxsuper);
void slu_symbfact_sizes(const void *h, int64_t *sizes);
/* xsup (nsupers+1 of n+1 written), supno / xlsub / xusub (n+1), lsub, usub */
void slu_symbfact_arrays(const void *h, int64_t *xsup, int64_t *supno, int64_t *xlsub,
                         int64_t *lsub, int64_t *xusub, int64_t *usub);
/* the same six arrays in place (valid until slu_symbfact_free): ptrs[0..5]
 * = xsup, supno, xlsub, lsub, xusub, usub (lengths as above) */
void slu_symbfact_views(const void *h, const int64_t **ptrs);
void slu_symbfact_free(void *h);
/* 1 when the last slu_symbfact / symbfact ran its countnz + fixupL epilogue
   (SRC/util.c:95-199) on the GPU (csrc/symbolic_dev.hip; SLU_SYMB_DEVICE=1
   forces it, =0 keeps it on the host; default: GPU for square problems with
   >= 20 000 supernodes when one is visible), 0 when on the host */
int slu_symbfact_last_epilogue_device(void);
/* Drop-in: the reference's own prototypes (SRC/superlu_defs.h:1079, 1091;
 * types in slu_abi.h).  A program linked against libslu_mi355x.so ahead of
 * the reference archive runs these in pdgssvx (SRC/pdgssvx.c:1046, 1075).
 * sp_colorder replaces SRC/sp_colorder.c:81 (AC's store and colbeg / colend
 * malloc'ed, rowind / nzval shared with A); symbfact replaces
 * SRC/symbfact.c:81 (xsup / supno and the Glu_freeable arrays malloc'ed,
 * freed by the reference's symbfact_SubFree / LU destructors), returning
 * -(lsub size) as the reference does. */
void sp_colorder(superlu_dist_options_t *options, SuperMatrix *A, int_t *perm_c,
                 int_t *etree, SuperMatrix *AC);
int_t symbfact(superlu_dist_options_t *options, int pnum, SuperMatrix *A, int_t *perm_c,
               int_t *etree, Glu_persist_t *Glu_persist, Glu_freeable_t *Glu_freeable);

/* Build this rank's LUstruct (dtype-typed dLUstruct_t/sLUstruct_t/zLUstruct_t
 * allocated by the library) holding P*A*P^T in the layout of
 * SRC/pddistribute.c, with ToRecv/ToSendD/ToSendR/bufmax filled as there. */
void *slu_distribute(const slu_symb *s, const slu_csc *A, int nprow,
                     int npcol, int myrow, int mycol);
void slu_lustruct_free(void *LUstruct, int dtype);
/* An LUstruct (freed by slu_lustruct_free) holding given arrays in the layout
 * pddistribute leaves (SRC/pddistribute.c:1283-1340, 1465-1493): flat index /
 * value arrays with offsets per local block column (Loff/Lvoff, nlc entries)
 * and block row (Uoff/Uvoff, nlr entries), -1 where the block column / row
 * is empty; ToSendR flattened nlc x npcol.  Used to feed the engine
 * LUstructs made by the reference's own front-end (tests/golden/refdump_*). */
void *slu_lustruct_build(int dtype, int64_t n, int64_t nsupers, const int_t *xsup,
                         const int_t *supno, int nprow, int npcol, const int_t *Lidx,
                         int64_t Lidx_cnt, const int64_t *Loff, const void *Lval,
                         int64_t Lval_cnt, const int64_t *Lvoff, const int_t *Uidx,
                         int64_t Uidx_cnt, const int64_t *Uoff, const void *Uval,
                         int64_t Uval_cnt, const int64_t *Uvoff, const int *ToRecv,
                         const int *ToSendD, const int *ToSendR, const int_t *bufmax);

/* The reference's structural pddistribute (the first-time
 * branch of SRC/pddistribute.c:673-1340, 1460-1509, ToRecv / ToSendD /
 * ToSendR :767-801, bufmax :2370 as the MAX over the whole grid): this rank's
 * LUstruct (freed by slu_lustruct_free) from the symbolic factorization
 * (xsup / supno of Glu_persist; xlsub / lsub / xusub / usub of Glu_freeable,
 * as symbfact leaves them) and A in the LUstruct's coordinates (CSC of
 * Pc Pr diag(R) A diag(C) Pc^T; every rank may pass all of A, entries of
 * other ranks' blocks are skipped).  Index arrays, block order and values
 * are the reference's bit for bit (tests/test_distribute.py).  NULL on error
 * (slu_last_error). */
void *slu_distribute_glu(int dtype, int64_t n, const int_t *xsup, const int_t *supno,
                         const int_t *xlsub, const int_t *lsub, const int_t *xusub,
                         const int_t *usub, const int64_t *xa, const int64_t *asub,
                         const void *a, int nprow, int npcol, int myrow, int mycol);

/* pddistribute's SamePattern_SameRowPerm branch on a library-built (or any
 * layout-compatible) LUstruct: zero its L / U values and drop in A's entries
 * (CSC in the LUstruct's coordinates, as slu_distribute_glu takes them). */
int slu_refill_values(int dtype, void *LUstruct, int64_t n, const int64_t *xa,
                      const int64_t *asub, const void *a, int nprow, int npcol,
                      int myrow, int mycol);

/* Permuted-matrix helpers for tests: B = P*A*P^T in CSC. */
slu_csc *slu_permute(const slu_csc *A, const int64_t *perm_c);

/* Flat view of a library-built LUstruct (contiguous *_dat arrays). */
typedef struct {
    int64_t nsupers;
    int_t *xsup, *supno;
    int_t *Lidx; int64_t Lidx_cnt; long *Lidx_off; /* Lrowind_bc_dat */
    void *Lval; int64_t Lval_cnt; long *Lval_off;   /* Lnzval_bc_dat */
    int_t *Uidx; int64_t Uidx_cnt; long *Uidx_off;  /* Ufstnz_br_dat */
    void *Uval; int64_t Uval_cnt; long *Uval_off;   /* Unzval_br_dat */
    int *ToRecv, *ToSendD, **ToSendR;
    int_t bufmax[5];
} slu_lu_view;
int slu_lu_get_view(void *LUstruct, int dtype, slu_lu_view *v);

#ifdef __cplusplus
}
#endif
#endif /* SLU_MI355X_H */
