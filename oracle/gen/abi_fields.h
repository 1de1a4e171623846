/* Field list shared by the reference-side probe (abi_probe.c, compiled against
 * /root/reference/SRC headers) and the mirror-side probe (tests compile it
 * against include/slu_abi.h).  Test infrastructure only. */
#define ABI_TYPES(X) X(gridinfo_t) X(superlu_scope_t) X(Glu_persist_t) \
  X(superlu_dist_options_t) X(SuperLUStat_t) X(dLocalLU_t) X(sLocalLU_t) \
  X(zLocalLU_t) X(dLUstruct_t) X(sLUstruct_t) X(zLUstruct_t) X(doublecomplex) \
  X(SuperMatrix) X(NCformat) X(NCPformat) X(Glu_freeable_t)
#define ABI_FIELDS(F) \
  F(gridinfo_t, comm) F(gridinfo_t, rscp) F(gridinfo_t, cscp) F(gridinfo_t, iam) \
  F(gridinfo_t, nprow) F(gridinfo_t, npcol) \
  F(superlu_dist_options_t, Fact) F(superlu_dist_options_t, ReplaceTinyPivot) \
  F(superlu_dist_options_t, lookahead_etree) F(superlu_dist_options_t, num_lookaheads) \
  F(superlu_dist_options_t, superlu_relax) F(superlu_dist_options_t, superlu_maxsup) \
  F(superlu_dist_options_t, superlu_n_gemm) F(superlu_dist_options_t, SymPattern) \
  F(superlu_dist_options_t, Algo3d) F(superlu_dist_options_t, ColPerm) \
  F(SuperMatrix, Stype) F(SuperMatrix, nrow) F(SuperMatrix, ncol) F(SuperMatrix, Store) \
  F(NCformat, nnz) F(NCformat, rowind) F(NCformat, colptr) \
  F(NCPformat, nnz) F(NCPformat, rowind) F(NCPformat, colbeg) F(NCPformat, colend) \
  F(Glu_freeable_t, lsub) F(Glu_freeable_t, xlsub) F(Glu_freeable_t, usub) \
  F(Glu_freeable_t, xusub) F(Glu_freeable_t, nzlmax) F(Glu_freeable_t, nzumax) \
  F(Glu_freeable_t, MemModel) F(Glu_freeable_t, nnzLU) \
  F(SuperLUStat_t, utime) F(SuperLUStat_t, ops) F(SuperLUStat_t, TinyPivots) \
  F(SuperLUStat_t, num_look_aheads) F(SuperLUStat_t, MaxActiveRTrees) \
  F(dLUstruct_t, Glu_persist) F(dLUstruct_t, Llu) F(dLUstruct_t, dt) \
  F(dLocalLU_t, Lrowind_bc_ptr) F(dLocalLU_t, Lnzval_bc_ptr) F(dLocalLU_t, Lnzval_bc_dat) \
  F(dLocalLU_t, Lnzval_bc_offset) F(dLocalLU_t, Unnz) F(dLocalLU_t, Ufstnz_br_ptr) \
  F(dLocalLU_t, Ufstnz_br_dat) F(dLocalLU_t, Unzval_br_ptr) F(dLocalLU_t, Unzval_br_dat) \
  F(dLocalLU_t, Unzval_br_offset) F(dLocalLU_t, Lsub_buf_2) F(dLocalLU_t, Uval_buf_2) \
  F(dLocalLU_t, ujrow) F(dLocalLU_t, bufmax) F(dLocalLU_t, ToRecv) F(dLocalLU_t, ToSendD) \
  F(dLocalLU_t, ToSendR) F(dLocalLU_t, ilsum) F(dLocalLU_t, ldalsum) F(dLocalLU_t, inv) \
  F(sLocalLU_t, Lnzval_bc_ptr) F(sLocalLU_t, Ufstnz_br_ptr) F(sLocalLU_t, Unzval_br_ptr) \
  F(sLocalLU_t, ujrow) F(sLocalLU_t, bufmax) F(sLocalLU_t, ToRecv) F(sLocalLU_t, ToSendR) \
  F(sLocalLU_t, inv) \
  F(zLocalLU_t, Lnzval_bc_ptr) F(zLocalLU_t, Ufstnz_br_ptr) F(zLocalLU_t, Unzval_br_ptr) \
  F(zLocalLU_t, ujrow) F(zLocalLU_t, bufmax) F(zLocalLU_t, ToRecv) F(zLocalLU_t, ToSendR) \
  F(zLocalLU_t, inv)
