/*
 * oracle_impl.h -- body of the CPU restatement of pdgstrf, instantiated once
 * per value type by oracle.c (d: double, s: float, z: doublecomplex).
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libslu_mi355x.so,
 * bench.py's measured leg) may call or link this.  It is the checker.
 *
 * The grid is simulated in one process: LU[p] is the LUstruct of rank
 * p = prow*Pc + pcol (SRC/superlu_defs.h:267 PNUM), each built exactly as the
 * reference's pddistribute lays it out.  The elimination visits supernodes in
 * natural order k = 0..nsupers-1; the reference visits them in the order of
 * its static schedule (SRC/dstatic_schedule.c:39), which is a topological
 * order of the same dependency DAG, so the factors agree up to the rounding
 * order of the Schur-complement sums.
 *
 * Expects: VT (value type), OR_NAME(x) (name mangling), LUS (LUstruct type),
 * and the scalar macros V_ZERO, V_SUB(a,b), V_MUL(a,b), V_DIV(a,b), V_ABS(a),
 * V_ISZERO(a), V_SET_THRESH(a,t) (keep sign), V_RECIP(a), and the flop
 * weights of the reference's stat->ops[FACT] accounting: F_SCALE(x), F_RANK1,
 * F_TRSM, F_SCHUR (SRC/pdgstrf2.c:252,262,318,355; SRC/pzgstrf2.c:253,263,319,356;
 * SRC/zlook_ahead_update.c:160).
 */

/* pdgstrf2_trsm, SRC/pdgstrf2.c:213-269 (diagonal block) and :302-355 (TRSM). */
static void OR_NAME(panel_l)(LUS **LU, int Pr, int Pc, int_t k, int_t *xsup,
                             int replace_tiny, double thresh, int *info_rank,
                             int *tiny, double *flops)
{
    int krow = (int)(k % Pr), kcol = (int)(k % Pc);
    int_t ljb = k / Pc;
    int_t fsupc = xsup[k], nsupc = xsup[k + 1] - xsup[k];
    /* --- diagonal process: unblocked LU of the nsupc x nsupc block --- */
    LUS *D = LU[krow * Pc + kcol];
    VT *lusup = D->Llu->Lnzval_bc_ptr[ljb];
    int_t nsupr = D->Llu->Lrowind_bc_ptr[ljb][1];
    for (int_t j = 0; j < nsupc; ++j) {
        VT *piv = &lusup[j + j * nsupr];
        if (replace_tiny && V_ABS(*piv) < thresh) {      /* SRC/pdgstrf2.c:217-232 */
            V_SET_THRESH(*piv, thresh);
            ++*tiny;
        }
        if (V_ISZERO(*piv)) {                             /* :246-247 */
            info_rank[krow * Pc + kcol] = (int)(fsupc + j + 1);
        } else {                                          /* :249-252 scale */
            VT temp = V_RECIP(*piv);
            for (int_t i = j + 1; i < nsupc; ++i)
                lusup[i + j * nsupr] = V_MUL(lusup[i + j * nsupr], temp);
            *flops += F_SCALE((double)(nsupc - j - 1));
        }
        /* rank-1 update inside the diagonal block, :256-263 (dger) */
        for (int_t l = j + 1; l < nsupc; ++l) {
            VT u = lusup[j + l * nsupr];
            for (int_t i = j + 1; i < nsupc; ++i)
                lusup[i + l * nsupr] = V_SUB(lusup[i + l * nsupr],
                                             V_MUL(lusup[i + j * nsupr], u));
        }
        *flops += F_RANK1 * (double)(nsupc - j - 1) * (double)(nsupc - j - 1);
    }
    /* --- L(:,k) := L(:,k) * U_kk^{-1} on every rank of process column kcol
     *     (dtrsm "R","U","N","N", :311 diag rank rows below the block,
     *     :352 other ranks all local rows) --- */
    for (int pr = 0; pr < Pr; ++pr) {
        LUS *R = LU[pr * Pc + kcol];
        int_t *index = R->Llu->Lrowind_bc_ptr[ljb];
        if (!index) continue;
        VT *X = R->Llu->Lnzval_bc_ptr[ljb];
        int_t ld = index[1];
        int_t r0 = (pr == krow) ? nsupc : 0;
        for (int_t i = r0; i < ld; ++i) {
            for (int_t j = 0; j < nsupc; ++j) {
                VT s = X[i + j * ld];
                for (int_t l = 0; l < j; ++l)
                    s = V_SUB(s, V_MUL(X[i + l * ld], lusup[l + j * nsupr]));
                X[i + j * ld] = V_DIV(s, lusup[j + j * nsupr]);
            }
        }
        *flops += F_TRSM * (double)nsupc * (nsupc + 1) * (double)(ld - r0);
    }
}

/* pdgstrs2_omp, SRC/pdgstrf2.c:761-900: U(k,:) segments := L_kk^{-1} seg. */
static void OR_NAME(panel_u)(LUS **LU, int Pr, int Pc, int_t k, int_t *xsup,
                             double *flops)
{
    int krow = (int)(k % Pr), kcol = (int)(k % Pc);
    int_t lk = k / Pr, ljb = k / Pc;
    int_t klst = xsup[k + 1], knsupc = xsup[k + 1] - xsup[k];
    LUS *D = LU[krow * Pc + kcol];
    VT *lusup = D->Llu->Lnzval_bc_ptr[ljb];
    int_t nsupr = D->Llu->Lrowind_bc_ptr[ljb][1];
    for (int pc = 0; pc < Pc; ++pc) {
        LUS *R = LU[krow * Pc + pc];
        int_t *usub = R->Llu->Ufstnz_br_ptr[lk];
        if (!usub) continue;
        VT *uval = R->Llu->Unzval_br_ptr[lk];
        int_t nb = usub[0], iukp = SLU_BR_HEADER, rukp = 0;
        for (int_t b = 0; b < nb; ++b) {
            int_t gb = usub[iukp];
            int_t nsupc = xsup[gb + 1] - xsup[gb];
            iukp += SLU_UB_DESCRIPTOR;
            for (int_t j = 0; j < nsupc; ++j) {
                int_t segsize = klst - usub[iukp++];
                if (!segsize) continue;
                /* dtrsv("L","N","U") on the trailing segsize part of L_kk */
                int_t off = knsupc - segsize;
                VT *x = &uval[rukp];
                for (int_t c = 0; c < segsize; ++c)
                    for (int_t r = c + 1; r < segsize; ++r)
                        x[r] = V_SUB(x[r], V_MUL(lusup[(off + r) + (off + c) * nsupr], x[c]));
                rukp += segsize;
                *flops += (double)segsize * (segsize + 1);
            }
        }
    }
}

/* Schur-complement update of step k on every rank: the GEMM of
 * SRC/dSchCompUdt-2Ddynamic.c:566-578 / dlook_ahead_update.c:163-169 followed by
 * dscatter_l (SRC/dscatter.c:110-189) and dscatter_u (:192-277). */
static void OR_NAME(schur)(LUS **LU, int Pr, int Pc, int_t k, int_t *xsup,
                           int_t *scratch_ind, double *flops)
{
    int krow = (int)(k % Pr), kcol = (int)(k % Pc);
    int_t fsupc = xsup[k], klst = xsup[k + 1];
    for (int pr = 0; pr < Pr; ++pr) {
        LUS *Ls = LU[pr * Pc + kcol];
        int_t *lsub = Ls->Llu->Lrowind_bc_ptr[k / Pc];
        if (!lsub) continue;
        VT *lusup = Ls->Llu->Lnzval_bc_ptr[k / Pc];
        int_t nsupr = lsub[1];
        for (int pc = 0; pc < Pc; ++pc) {
            LUS *Us = LU[krow * Pc + pc];
            int_t *usub = Us->Llu->Ufstnz_br_ptr[k / Pr];
            if (!usub) continue;
            VT *uval = Us->Llu->Unzval_br_ptr[k / Pr];
            LUS *Dst = LU[pr * Pc + pc];
            /* walk L blocks of column k in process row pr */
            int_t nlb = lsub[0], lptr = SLU_BC_HEADER, luptr = 0;
            for (int_t lb = 0; lb < nlb; ++lb) {
                int_t ib = lsub[lptr], nbrow = lsub[lptr + 1];
                int_t *rows = &lsub[lptr + SLU_LB_DESCRIPTOR];
                if (ib != k) {
                    /* walk U blocks of row k in process column pc */
                    int_t nub = usub[0], iukp = SLU_BR_HEADER, rukp = 0;
                    for (int_t ub = 0; ub < nub; ++ub) {
                        int_t jb = usub[iukp];
                        int_t nsupc = xsup[jb + 1] - xsup[jb];
                        int_t *fst = &usub[iukp + SLU_UB_DESCRIPTOR];
                        if (ib >= jb) {
                            /* dscatter_l: locate L(ib,jb) in column jb (linear
                             * search, :137-142), indirect row map (:156-169) */
                            int_t *index = Dst->Llu->Lrowind_bc_ptr[jb / Pc];
                            int_t ldv = index[1], lptrj = SLU_BC_HEADER, luptrj = 0;
                            while (index[lptrj] != ib) {
                                luptrj += index[lptrj + 1];
                                lptrj += SLU_LB_DESCRIPTOR + index[lptrj + 1];
                            }
                            int_t dnb = index[lptrj + 1];
                            int_t fnz = xsup[ib];
                            for (int_t i = 0; i < dnb; ++i)
                                scratch_ind[index[lptrj + SLU_LB_DESCRIPTOR + i] - fnz] = i;
                            VT *nzval = Dst->Llu->Lnzval_bc_ptr[jb / Pc] + luptrj;
                            int_t ruk = rukp;
                            for (int_t jj = 0; jj < nsupc; ++jj) {
                                int_t seg = klst - fst[jj];
                                if (!seg) continue;
                                for (int_t i = 0; i < nbrow; ++i) {
                                    VT s = V_ZERO;
                                    int_t r = luptr + i;
                                    for (int_t t = 0; t < seg; ++t)
                                        s = V_ADD(s, V_MUL(lusup[r + (fst[jj] - fsupc + t) * nsupr],
                                                           uval[ruk + t]));
                                    int_t d = scratch_ind[rows[i] - fnz];
                                    nzval[d + jj * ldv] = V_SUB(nzval[d + jj * ldv], s);
                                }
                                ruk += seg;
                                *flops += F_SCHUR * nbrow * seg;
                            }
                        } else {
                            /* dscatter_u: locate U(ib,jb) in block row ib
                             * (:229-235), per column segment (:240-272) */
                            int_t *index = Dst->Llu->Ufstnz_br_ptr[ib / Pr];
                            VT *ucolbase = Dst->Llu->Unzval_br_ptr[ib / Pr];
                            int_t ilst = xsup[ib + 1];
                            int_t iuip = SLU_BR_HEADER, ruip = 0;
                            while (index[iuip] < jb) {
                                ruip += index[iuip + 1];
                                iuip += SLU_UB_DESCRIPTOR + (xsup[index[iuip] + 1] - xsup[index[iuip]]);
                            }
                            iuip += SLU_UB_DESCRIPTOR;
                            int_t ruk = rukp;
                            for (int_t jj = 0; jj < nsupc; ++jj) {
                                int_t seg = klst - fst[jj];
                                int_t dfnz = index[iuip + jj];
                                if (seg) {
                                    VT *ucol = &ucolbase[ruip];
                                    for (int_t i = 0; i < nbrow; ++i) {
                                        VT s = V_ZERO;
                                        int_t r = luptr + i;
                                        for (int_t t = 0; t < seg; ++t)
                                            s = V_ADD(s, V_MUL(lusup[r + (fst[jj] - fsupc + t) * nsupr],
                                                               uval[ruk + t]));
                                        int_t rel = rows[i] - dfnz;
                                        ucol[rel] = V_SUB(ucol[rel], s);
                                    }
                                    ruk += seg;
                                    *flops += F_SCHUR * nbrow * seg;
                                }
                                ruip += ilst - dfnz;
                            }
                        }
                        /* advance to the next U block */
                        for (int_t jj = 0; jj < nsupc; ++jj) rukp += klst - fst[jj];
                        iukp += SLU_UB_DESCRIPTOR + nsupc;
                    }
                }
                lptr += SLU_LB_DESCRIPTOR + nbrow;
                luptr += nbrow;
            }
        }
    }
}

/* The whole factorization; see the file header. */
int OR_NAME(factor)(int Pr, int Pc, void **LUv, int n, int replace_tiny,
                    double anorm, int *info, int *tiny, double *flops)
{
    LUS **LU = (LUS **)LUv;
    int_t *xsup = LU[0]->Glu_persist->xsup;
    int_t *supno = LU[0]->Glu_persist->supno;
    int_t nsupers = supno[n - 1] + 1;
    double thresh = (double)FLT_EPSILON * 0.5 * anorm; /* smach_dist("Epsilon")*anorm, SRC/pdgstrf.c:412-413 */
    int_t *scratch = (int_t *)malloc(sizeof(int_t) * 1024);
    int *info_rank = (int *)calloc(Pr * Pc, sizeof(int));
    *tiny = 0;
    *flops = 0.0;
    for (int_t k = 0; k < nsupers; ++k) {
        int_t w = xsup[k + 1] - xsup[k];
        if (w > 1024) { free(scratch); return -1; }
        OR_NAME(panel_l)(LU, Pr, Pc, k, xsup, replace_tiny, thresh, info_rank, tiny, flops);
        OR_NAME(panel_u)(LU, Pr, Pc, k, xsup, flops);
        OR_NAME(schur)(LU, Pr, Pc, k, xsup, scratch, flops);
    }
    /* MIN over ranks of the per-rank info (n+1 when none), SRC/pdgstrf.c:1927-1931 */
    int mn = n + 1;
    for (int p = 0; p < Pr * Pc; ++p)
        if (info_rank[p] && info_rank[p] < mn) mn = info_rank[p];
    *info = (mn == n + 1) ? 0 : mn;
    free(info_rank);
    free(scratch);
    return 0;
}
