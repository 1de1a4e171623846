// Device epilogue of symbfact: the reference's countnz
// and fixupL (SRC/util.c:95-152, 163-199), which symbfact runs after its
// search (SRC/symbfact.c:181-186), on the GPU.  HBM-bound integer work:
//
//   fixupL   every supernode keeps its first column's subscript list, copied
//            into one compact lsub in supernode order, rows past min(m, n)
//            mapped to EMPTY (the reference applies perm_r there: the
//            identity on pivoted rows); xlsub of a supernode's first column
//            = the list's offset, of its other columns = the offset past it
//   countnz  nnzL = sum over supernodes of w*len - w(w-1)/2, nnzU = the
//            diagonal blocks' w(w+1)/2 plus, per U segment first row f,
//            xsup[supno[f]+1] - f
//
// The search itself (csrc/symbolic.cpp) stays on the host: its depth-first
// order decides the subscripts' order and is inherently sequential.  The
// results are the host epilogue's bit for bit (tests/test_symbolic.py, GPU:
// every symb_* golden of the reference through this path).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "noinit_vec.h"

namespace slu {
namespace symbdev {

using I = int64_t;

#define SDCHK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            err = std::string(#x) + ": " + hipGetErrorString(e_);                                  \
            return false;                                                                          \
        }                                                                                          \
    } while (0)

// one workgroup per supernode (grid-stride): its first list into the
// compact lsub; the supernode's nnzL / diagonal-block nnzU terms
__global__ void __launch_bounds__(256) k_fixup(const int32_t *raw, const I *src, const I *off, const int32_t *xsup,
                                               I nsup, I mn, I *out, unsigned long long *cnt) {
    for (I s = blockIdx.x; s < nsup; s += gridDim.x) {
        const I a = src[s], o = off[s], len = off[s + 1] - o;
        for (I i = threadIdx.x; i < len; i += blockDim.x) {
            const int32_t r = raw[a + i];
            out[o + i] = r < mn ? (I)r : (I)-1;
        }
        if (threadIdx.x == 0) {
            const I w = xsup[s + 1] - xsup[s];
            atomicAdd(&cnt[0], (unsigned long long)(w * len - w * (w - 1) / 2));
            atomicAdd(&cnt[1], (unsigned long long)(w * (w + 1) / 2));
        }
    }
}

// xlsub of every column from its supernode's offsets
__global__ void __launch_bounds__(256) k_xlsub(const int32_t *supno, const int32_t *xsup, const I *off, I n, I *xl) {
    const I c = (I)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const int32_t s = supno[c];
    xl[c] = c == xsup[s] ? off[s] : off[s + 1];
}

// the U segments' nnzU terms, block-reduced, one atomic per workgroup
__global__ void __launch_bounds__(256) k_usub(const int32_t *usub, I nu, const int32_t *supno, const int32_t *xsup,
                                              unsigned long long *cnt) {
    __shared__ unsigned long long part[4];
    unsigned long long acc = 0;
    for (I p = (I)blockIdx.x * blockDim.x + threadIdx.x; p < nu; p += (I)gridDim.x * blockDim.x) {
        const int32_t f = usub[p];
        acc += (unsigned long long)(xsup[supno[f] + 1] - f);
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(&cnt[1], part[0] + part[1] + part[2] + part[3]);
}

template <class T> struct Dev {
    T *p = nullptr;
    ~Dev() {
        if (p) (void)hipFree(p);
    }
};

// n x n (m = n): raw = the search's lsub (first and last lists per
// supernode, xlsub_raw positions), xsup / supno / usub int32.  Fills lsub
// (compact, the final size known from the lists), xlsub[0..n], nnzL / nnzU.
bool epilogue(I n, I nsup, const int32_t *raw, I raw_len, const I *xlsub_raw, const int32_t *xsup,
              const int32_t *supno, const int32_t *usub, I nu, i64_vec &lsub, std::vector<I> &xlsub,
              I *nnzL, I *nnzU, std::string &err) {
    // per supernode: source position and compact offset (host: O(nsup))
    std::vector<I> src(nsup), off(nsup + 1);
    off[0] = 0;
    for (I s = 0; s < nsup; ++s) {
        const I f = xsup[s];
        src[s] = xlsub_raw[f];
        off[s + 1] = off[s] + (xlsub_raw[f + 1] - xlsub_raw[f]);
    }
    const I total = off[nsup];
    lsub.resize(total);
    // one process per GPU: the device of this process's local rank, as the
    // factorization picks it (abi.cpp pick_device)
    {
        int nd = 0;
        const char *e = getenv("SUPERLU_DEVICE");
        const char *lr = getenv("MPI_LOCALRANKID");
        if (!lr) lr = getenv("OMPI_COMM_WORLD_LOCAL_RANK");
        if (!lr) lr = getenv("LOCAL_RANK");
        if ((e || lr) && hipGetDeviceCount(&nd) == hipSuccess && nd > 0)
            SDCHK(hipSetDevice(e ? atoi(e) : atoi(lr) % nd));
    }
    xlsub.resize(n + 1);
    Dev<int32_t> d_raw, d_xsup, d_supno, d_usub;
    Dev<I> d_src, d_off, d_out, d_xl;
    Dev<unsigned long long> d_cnt;
    SDCHK(hipMalloc(&d_raw.p, std::max<I>(raw_len, 1) * 4));
    SDCHK(hipMalloc(&d_xsup.p, (nsup + 1) * 4));
    SDCHK(hipMalloc(&d_supno.p, (n + 1) * 4));
    SDCHK(hipMalloc(&d_usub.p, std::max<I>(nu, 1) * 4));
    SDCHK(hipMalloc(&d_src.p, std::max<I>(nsup, 1) * 8));
    SDCHK(hipMalloc(&d_off.p, (nsup + 1) * 8));
    SDCHK(hipMalloc(&d_out.p, std::max<I>(total, 1) * 8));
    SDCHK(hipMalloc(&d_xl.p, (n + 1) * 8));
    SDCHK(hipMalloc(&d_cnt.p, 2 * sizeof(unsigned long long)));
    SDCHK(hipMemcpy(d_raw.p, raw, raw_len * 4, hipMemcpyHostToDevice));
    SDCHK(hipMemcpy(d_xsup.p, xsup, (nsup + 1) * 4, hipMemcpyHostToDevice));
    SDCHK(hipMemcpy(d_supno.p, supno, (n + 1) * 4, hipMemcpyHostToDevice));
    if (nu) SDCHK(hipMemcpy(d_usub.p, usub, nu * 4, hipMemcpyHostToDevice));
    SDCHK(hipMemcpy(d_src.p, src.data(), nsup * 8, hipMemcpyHostToDevice));
    SDCHK(hipMemcpy(d_off.p, off.data(), (nsup + 1) * 8, hipMemcpyHostToDevice));
    SDCHK(hipMemset(d_cnt.p, 0, 2 * sizeof(unsigned long long)));
    const int gb = (int)std::min<I>(std::max<I>(nsup, 1), 8192);
    hipLaunchKernelGGL(k_fixup, dim3(gb), dim3(256), 0, 0, d_raw.p, d_src.p, d_off.p, d_xsup.p, nsup, n, d_out.p,
                       d_cnt.p);
    hipLaunchKernelGGL(k_xlsub, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, d_supno.p, d_xsup.p, d_off.p,
                       n, d_xl.p);
    if (nu)
        hipLaunchKernelGGL(k_usub, dim3((unsigned)std::min<I>((nu + 255) / 256, 4096)), dim3(256), 0, 0, d_usub.p,
                           nu, d_supno.p, d_xsup.p, d_cnt.p);
    SDCHK(hipGetLastError());
    unsigned long long cnt[2];
    SDCHK(hipMemcpy(lsub.data(), d_out.p, total * 8, hipMemcpyDeviceToHost));
    SDCHK(hipMemcpy(xlsub.data(), d_xl.p, n * 8, hipMemcpyDeviceToHost));
    SDCHK(hipMemcpy(cnt, d_cnt.p, sizeof cnt, hipMemcpyDeviceToHost));
    xlsub[n] = total;
    *nnzL = (I)cnt[0];
    *nnzU = (I)cnt[1];
    return true;
}

} // namespace symbdev
} // namespace slu

// C++ entry for csrc/symbolic.cpp (the full library links both)
bool slu_symb_epilogue_dev(int64_t n, int64_t nsup, const int32_t *raw, int64_t raw_len, const int64_t *xlsub_raw,
                           const int32_t *xsup, const int32_t *supno, const int32_t *usub, int64_t nu,
                           slu::i64_vec &lsub, std::vector<int64_t> &xlsub, int64_t *nnzL, int64_t *nnzU,
                           std::string &err) {
    return slu::symbdev::epilogue(n, nsup, raw, raw_len, xlsub_raw, xsup, supno, usub, nu, lsub, xlsub, nnzL, nnzU,
                                  err);
}

bool slu_symb_have_device() {
    int nd = 0;
    return hipGetDeviceCount(&nd) == hipSuccess && nd > 0;
}
