/*
 * krylov_amd.h -- C ABI of the MI355X-native Krylov inner loop.
 *
 * This is the drop-in boundary for the reference's GPU solver families
 * (5enxia/parallel-krylov, v3/gpu and v3/gpu/mpi). The reference binds its
 * device work through cupy (cuBLAS ddot, cuSPARSE csrmv, elementwise ufuncs)
 * and its communication through mpi4py; every entry point below names the
 * reference interface it replaces (file:line under the reference tree).
 *
 * Conventions
 *  - Plain pointers and sizes only; no torch or HIP types in signatures.
 *    `stream` arguments are a hipStream_t passed as void* (NULL = default).
 *  - Every function returns KR_OK (0) or a negative KR_ERR_* code; the
 *    message of the last failure on the calling thread is kr_last_error().
 *    Nothing throws across the ABI.
 *  - All vectors and matrices are fp64 values with int32 column indices;
 *    row pointers are int32 or int64 (flag `rowptr64`).
 *  - Device pointers are "dev"; host pointers are "host".
 */
#ifndef KRYLOV_AMD_H
#define KRYLOV_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KR_OK 0
#define KR_ERR_INVALID -1 /* bad argument / shape */
#define KR_ERR_HIP -2     /* HIP runtime failure */
#define KR_ERR_RCCL -3    /* RCCL failure */
#define KR_ERR_NOMEM -4   /* device allocation failed */
#define KR_ERR_STATE -5   /* call out of order (e.g. step before begin) */

/* Solver methods (reference modules v3/gpu/{cg,mrr,kskipcg,kskipmrr,adaptivekskipmrr}.py). */
#define KR_METHOD_CG 0
#define KR_METHOD_MRR 1
#define KR_METHOD_KSKIPCG 2
#define KR_METHOD_KSKIPMRR 3
#define KR_METHOD_ADAPTIVE_KSKIPMRR 4
/* Preconditioned and pipelined CG (reference v1/threads/pipeline/{pcg,
 * chronopoulos_gear,gropp,pipeline}.py: `method(A, b, ilu, epsilon, T, pt)`),
 * restated as the textbook algorithms those files name with a Jacobi
 * (kr_solve_set_precond) or ILU (kr_solve_set_precond_ilu) preconditioner
 * (DESIGN.md §5b). maxiter < 0 means
 * 2N (v1/threads/common.py:47); iterations i = 1 .. maxiter-1. */
#define KR_METHOD_PCG 5
#define KR_METHOD_CG_GEAR 6
#define KR_METHOD_GROPP 7
#define KR_METHOD_PIPECG 8

/* Library identification. kr_version() returns KR_ABI_VERSION; a binding
 * checks it before it uses any struct below (INTEGRATION.md "ABI versions").
 *   100  round 1
 *   200  kr_solve_params gained nan_guard and kr_solve_result diverged (both
 *        structs changed size); maxiter = 0 is honoured instead of meaning
 *        the default (CG / k-skip CG return r0, the MrR family is refused).
 *   201  kr_solve_set_precond_ilu added (no struct or behaviour change).
 *   202  kr_system_shard_code_patterns added (no struct or behaviour change).
 *   203  kr_system_shard_dia_full_blocks added (no struct or behaviour change).
 *   204  kr_solve_kernel_stats reports device windows over a device's shards.
 *   205  kr_system_shard_box added (no struct or behaviour change). */
#define KR_ABI_VERSION 205
int kr_version(void);
const char* kr_last_error(void);
/* Number of HIP devices visible to this process (0 when none). */
int kr_device_count(int* count);

/* ------------------------------------------------------------------------
 * Primitive kernels (async on `stream`; operands on one device).
 * ------------------------------------------------------------------------ */

/* y[i] = sum_j val[j] * x[col[j]] over row i, summed sequentially in stored
 * order without FMA contraction (bitwise equal to scipy's csr_matvec).
 * Replaces cupyx csr_matrix.dot called at v3/gpu/common.py:119 and
 * v3/gpu/mpi/common.py:150. `x` is indexed by `col` directly. */
int kr_spmv_csr_f64(const void* rowptr_dev, int rowptr64, const int32_t* col_dev,
                    const double* val_dev, int64_t n_rows, const double* x_dev,
                    double* y_dev, void* stream);

/* Two right-hand sides in one pass over A: y1 = A x1, y2 = A x2 (each row
 * summed as in kr_spmv_csr_f64). Replaces the pairs of MultiGpu.dot calls of
 * the k-skip basis loops (v3/gpu/kskipmrr.py:47-50, v3/gpu/kskipcg.py:39-42). */
int kr_spmv2_csr_f64(const void* rowptr_dev, int rowptr64, const int32_t* col_dev,
                     const double* val_dev, int64_t n_rows, const double* x1_dev,
                     const double* x2_dev, double* y1_dev, double* y2_dev, void* stream);

/* *out_dev = <u, v>, deterministic two-stage reduction.
 * Replaces cupy.dot (cuBLAS ddot), e.g. v3/gpu/cg.py:32. */
int kr_dot_f64(const double* u_dev, const double* v_dev, int64_t n, double* out_dev,
               void* stream);

/* out_dev[0..count) = Gram coefficients of `count` vector pairs
 * (u_ptrs[i], v_ptrs[i]) in ONE pass over the distinct vectors.
 * Replaces the 6k+5 cupy.dot calls of v3/gpu/kskipmrr.py:53-61 and the 6k+7 of
 * v3/gpu/kskipcg.py:44-52. count <= 64. */
int kr_multidot_f64(const double* const* u_ptrs_host, const double* const* v_ptrs_host,
                    int count, int64_t n, double* out_dev, void* stream);

/* *out_dev = ||u||_2 = sqrt(<u, u>) (same reduction as kr_dot_f64).
 * Replaces cupy.linalg.norm, e.g. v3/gpu/kskipmrr.py:26,42 and v3/gpu/common.py:33. */
int kr_norm2_f64(const double* u_dev, int64_t n, double* out_dev, void* stream);

/* k-skip MrR Gram coefficients (v3/gpu/kskipmrr.py:53-61) of the basis rows
 * Ar[0..k+1] and Ay[0..k], row m at ar_dev + m*ld (ld >= n):
 *   out[0 .. 2k+3)            alpha[j] = <Ar[j/2], Ar[j/2 + j%2]>
 *   out[2k+3 .. 4k+5)         beta[j]  = <Ay[j/2], Ar[j/2 + j%2]>, beta[0] = 0
 *   out[4k+5 .. 6k+6)         delta[j] = <Ay[j/2], Ay[j/2 + j%2]>
 * i.e. the 6k+5 dots plus beta[0], laid out as the alpha/beta/delta arrays
 * kr_kskipmrr_recurrence takes. The solver engine fuses these products into
 * the basis SpMVs instead; this entry point serves callers with their own basis. */
int kr_gram_kskipmrr_f64(const double* ar_dev, const double* ay_dev, int k, int64_t n,
                         int64_t ld, double* out_dev, void* stream);

/* k-skip CG Gram coefficients (v3/gpu/kskipcg.py:44-52) of Ar[0..k], Ap[0..k+1]:
 *   out[0 .. 2k+1)            a[j] = <Ar[j/2], Ar[j/2 + j%2]>
 *   out[2k+1 .. 4k+5)         f[j] = <Ap[j/2], Ap[j/2 + j%2]>, f[2k+3] = 0
 *                             (the reference dots with the never-computed Ap[k+2])
 *   out[4k+5 .. 6k+7)         c[j] = <Ar[j/2], Ap[j/2 + j%2]>                     */
int kr_gram_kskipcg_f64(const double* ar_dev, const double* ap_dev, int k, int64_t n,
                        int64_t ld, double* out_dev, void* stream);

/* Fused k-skip MrR / MrR vector step (v3/gpu/kskipmrr.py:67-71):
 *   y = eta*y + zeta*ar1 ; z = eta*z - zeta*r ; r -= y ; x -= z
 * rounded exactly like the numpy statements (no FMA). first != 0 selects the
 * initial step (v3/gpu/kskipmrr.py:30-33): y = zeta*ar1 ; z = (-zeta)*r. */
int kr_update_mrr_f64(double eta, double zeta, int first, double* y_dev,
                      const double* ar1_dev, double* z_dev, double* r_dev,
                      double* x_dev, int64_t n, void* stream);

/* Fused CG vector step (v3/gpu/cg.py:34-35): x += alpha*p ; r -= alpha*v. */
int kr_update_cg_f64(double alpha, double* x_dev, const double* p_dev, double* r_dev,
                     const double* v_dev, int64_t n, void* stream);

/* Host scalar recurrences, statement-for-statement with the reference
 * (libm pow for `**2`, left-to-right, no FMA). They take and return the Gram
 * coefficient arrays exactly as the reference holds them.
 *
 * k-skip MrR (v3/gpu/kskipmrr.py:64-66, 74-90): given alpha[2k+3],
 * beta[2k+2], delta[2k+1] from the basis, writes zeta[k+1], eta[k+1] for
 * the k+1 vector steps of one outer iteration (arrays are consumed). */
int kr_kskipmrr_recurrence(int k, double* alpha, double* beta, double* delta,
                           double* zeta_out, double* eta_out);
/* k-skip CG (v3/gpu/kskipcg.py:55-56, 64-72): a[2k+2], f[2k+4], c[2k+2] in,
 * alpha[k+1], beta[k+1] out (arrays are consumed). */
int kr_kskipcg_recurrence(int k, double* a, double* f, double* c, double* alpha_out,
                          double* beta_out);

/* ------------------------------------------------------------------------
 * Communicator (replaces mpi4py comm.Allgather on the hot path,
 * v3/gpu/mpi/common.py:163, and the P2P copies of v3/gpu/common.py:117,122).
 * RCCL over xGMI, one rank per GPU.
 * ------------------------------------------------------------------------ */
typedef struct kr_comm kr_comm;
#define KR_UNIQUE_ID_BYTES 128
/* Rank 0 creates the id; the caller broadcasts it (e.g. torch.distributed). */
int kr_comm_unique_id(uint8_t* id_out /* KR_UNIQUE_ID_BYTES */);
int kr_comm_init(kr_comm** comm, const uint8_t* id, int nranks, int rank, int device);
int kr_comm_destroy(kr_comm* comm);

/* In-place sum over the ranks of buf_dev[0..count) (ncclAllReduce). Replaces
 * the Allgather + host sum of the reference's distributed dots
 * (v3/gpu/mpi/common.py:163). The solver engine all-gathers the per-rank
 * partials instead and sums them in rank order (deterministic histories). */
int kr_allreduce_sum_f64(kr_comm* comm, double* buf_dev, int64_t count, void* stream);

/* Halo exchange of one halo-extended vector x_dev: pieces are (peer, first
 * element of x_dev, count) triples, nsend sent and nrecv received in one RCCL
 * group (ncclSend/ncclRecv). The element offsets are local: global row g of a
 * kr_halo_plan piece lives at g - row0 + pad in the System layout. Replaces
 * the full-vector broadcast + gather of MultiGpu.dot (v3/gpu/common.py:115-122,
 * v3/gpu/mpi/common.py:154-163). */
int kr_halo_exchange_f64(kr_comm* comm, double* x_dev, const int64_t* recv, int nrecv,
                         const int64_t* send, int nsend, void* stream);

/* ------------------------------------------------------------------------
 * Distributed system: A and every vector row-partitioned into contiguous
 * shards (replaces MultiGpu.init/alloc, v3/gpu/common.py:62-109 and
 * v3/gpu/mpi/common.py:73-134). A process owns `nshards` shards. Without a
 * communicator they are the whole system; with one, every rank owns its
 * shards (1..16, e.g. the GPU_IDS range of MultiGpu.alloc,
 * v3/gpu/mpi/common.py:100-118), global shards are numbered rank after rank,
 * halo pieces between two shards of one rank are device copies and the
 * others RCCL send/recv; dot products are summed in global shard order
 * either way, so a partition gives the same bits in one process or over
 * ranks.
 * ------------------------------------------------------------------------ */
typedef struct kr_system kr_system;

/* row_begin[0..nshards] are GLOBAL row offsets of this process's shards
 * (contiguous, increasing; with a communicator, rank r's block follows rank
 * r-1's). devices[s] is the HIP device of shard s. Collective over `comm`. */
int kr_system_create(kr_system** sys, int64_t n_global, int nshards, const int* devices,
                     const int64_t* row_begin, kr_comm* comm);
int kr_system_destroy(kr_system* sys);

/* Adopt a CSR block already resident on the shard's device: rows
 * row_begin[s]..row_begin[s+1], GLOBAL column indices, rowptr starting at
 * rowptr[0] (need not be 0). The caller keeps the buffers alive until
 * kr_system_destroy; column indices are rewritten IN PLACE to the shard's
 * local (halo-extended) numbering by kr_system_finalize.
 * The matrix is FROZEN at kr_system_finalize: the SpMV kernels stream derived
 * copies built there (offset masks from the columns, the value dictionary's
 * codes and table, diagonal-offset values), so values changed in val_dev
 * after finalize are seen by some kernels and not by others. To solve with
 * new values, create (adopt, finalize) a new system. */
int kr_system_adopt_csr(kr_system* sys, int shard, const void* rowptr_dev, int rowptr64,
                        int32_t* col_dev, const double* val_dev);

/* Adopt a DENSE row block already resident on the shard's device: rows
 * row_begin[s]..row_begin[s+1] of A as a row-major (n_local x n_global)
 * float64 array with leading dimension ld >= n_global (global columns).
 * Replaces the reference's np.ndarray branch of MultiGpu.alloc
 * (v3/gpu/common.py:100-101, v3/gpu/mpi/common.py:124-125), whose product is
 * a cuBLAS dgemv; here a wave-per-row GEMV with the same fused epilogues as
 * the SpMV. The caller keeps the buffer alive until kr_system_destroy. */
int kr_system_adopt_dense(kr_system* sys, int shard, const double* a_dev, int64_t ld);

/* Generate this shard's rows of a synthetic SPD matrix on the device.
 * dim = 2 or 3: 5-/7-point Poisson on an n_side^dim grid, lexicographic
 * order, diagonal 2*dim, off-diagonals -1 (scipy kronsum of tridiag(-1,2,-1));
 * when n_global = n_side^(dim-1) * nz with nz != n_side, the same operator on
 * a box of nz planes (e.g. the slab one rank of a multi-GPU cube owns).
 * Banded: h distinct offsets in [1,W] drawn from `seed`, a(i,i+-o) = -u,
 * diagonal = sum|off| + 1 (see DESIGN.md for the exact definition). */
int kr_system_gen_poisson(kr_system* sys, int dim, int64_t n_side);
int kr_system_gen_banded(kr_system* sys, int h, int64_t width, uint64_t seed,
                         int rowptr64);
/* Column remap, halo plan, row blocks and workspaces. Call once after the
 * matrix of every shard is set. */
int kr_system_finalize(kr_system* sys);
/* Device CSR arrays of shard s (after finalize: LOCAL column numbering, own
 * row r of the halo-extended vector sits at index pad + r; see shard_info). */
int kr_system_csr(kr_system* sys, int shard, const void** rowptr_dev, int* rowptr64,
                  const int32_t** col_dev, const double** val_dev, int64_t* pad);
/* Info: n_local, halo_lo, halo_hi, nnz of shard s. */
int kr_system_shard_info(kr_system* sys, int shard, int64_t* n_local, int64_t* halo_lo,
                         int64_t* halo_hi, int64_t* nnz);
/* Storage layout the SpMV uses for shard s (after finalize): mask_bits = 0
 * for plain CSR columns, else 8/16/32/64 when every row's columns are
 * row + offsets[b] for the set bits b of a per-row mask over n_offsets
 * distinct offsets (stencil/banded matrices; the column array is then not
 * read). interior_lo/hi: rows whose columns need no halo (the part of the
 * SpMV that overlaps the exchange). Pointers may be NULL. */
int kr_system_shard_layout(kr_system* sys, int shard, int* mask_bits, int* n_offsets,
                           int64_t* interior_lo, int64_t* interior_hi);
/* Value storage the row-walk SpMV uses for shard s (after finalize):
 * dict_values = 0 for the 8-byte value stream, else the number (<= 256) of
 * distinct value bit patterns, each entry then streamed as a 1-byte code into
 * that table (lossless; short-row CSR blocks such as stencils; KR_VDICT=0
 * disables). Replaces nothing in the reference: the cuSPARSE csrmv behind
 * v3/gpu/common.py:119 always streams 8-byte values. */
int kr_system_shard_values(kr_system* sys, int shard, int* dict_values);
/* Stencil code width of shard s (after finalize): 0 when the stencil SpMV
 * does not serve the shard, else the bits per slot code (8: one uint64 per
 * row; 4 / 2: one uint32 / uint16 per row, for dictionaries of <= 15 / <= 3
 * values on the 7-point pattern), i.e. the bytes of A one row streams.
 * Replaces nothing in the reference (cuSPARSE csrmv streams CSR). */
int kr_system_shard_codes(kr_system* sys, int shard, int* code_bits);
/* Stencil code patterns of shard s (after finalize): 0 when the stencil
 * SpMV streams its codes per row, else the number (<= 256) of distinct
 * 512-row code blocks; each is stored once and every row block holds one
 * 4-byte pattern id, so the walk reads its codes from that small table (L2)
 * instead of code_bits bytes per row (a constant-coefficient stencil on a
 * box: 9 blocks at 512^3). Lossless, compared byte for byte at finalize;
 * KR_STENCIL_PATTERNS=0 disables. Replaces nothing in the reference. */
int kr_system_shard_code_patterns(kr_system* sys, int shard, int* patterns);
/* Box stencil of shard s (after finalize): 1 when the shard is a constant-
 * coefficient 7-point stencil on an n = 512 box (offsets -W, -512, -1, 0,
 * +1, +512, +W; every entry of an offset the same finite value; absent
 * entries exactly the box faces -- checked on the code patterns), else 0.
 * Such a shard's k-skip basis pairs can run matrix-free (the box pair,
 * kr_pair.hip: the absent operands read as 0.0, bitwise the CSR rows).
 * KR_BOX=0 disables. Replaces nothing in the reference. */
int kr_system_shard_box(kr_system* sys, int shard, int* box);
/* Full-block run of shard s's symmetric DIA walk (after finalize): the
 * longest run of 256-row blocks [first, first + count) that are whole and
 * whose rows hold every offset (a band matrix: all but its first and last
 * blocks). The walk does not load their offset masks (all ones); count = 0
 * when the shard has no DIA walk. KR_DIAW_FULLRUN=0 disables. Replaces
 * nothing in the reference. */
int kr_system_shard_dia_full_blocks(kr_system* sys, int shard, int64_t* first, int64_t* count);
/* Symmetric diagonal-offset values of shard s (after finalize): 1 when the
 * shard's offsets and stored values are symmetric (checked bitwise at
 * finalize) and the DIA SpMV reads each lower entry as the mirrored upper
 * entry of an earlier row, which the workgroup of that row block streams at
 * the same time: only the upper half and the diagonal come from HBM (KR_DIA_SYM=0
 * disables). Same values, same summation order: the results do not change.
 * Replaces nothing in the reference (cuSPARSE csrmv streams every value). */
int kr_system_shard_dia_sym(kr_system* sys, int shard, int* sym);
/* Launch geometry of shard s (after finalize): grid = workgroups of the
 * elementwise kernels, spmv_grid = workgroups of the SpMV kernels,
 * stencil_walk = 0 for the row-walk SpMV (256-row blocks, one row per lane)
 * or P > 0 for the stencil SpMV (512-row blocks, two rows per lane, walking
 * P blocks per step). Together with the interior range of
 * kr_system_shard_layout they fix the summation order of every dot product
 * (oracle/gpu_order.py restates it for the bitwise GPU-order parity tests).
 * Replaces nothing in the reference (cuBLAS ddot's order is internal).
 * format = KR_FORMAT_*. Pointers may be NULL. */
int kr_system_shard_sched(kr_system* sys, int shard, int* grid, int* spmv_grid,
                          int* stencil_walk, int* format);
/* kr_system_shard_sched format: the SpMV kernel family serving the shard. */
#define KR_FORMAT_CSR 0     /* row walk over CSR (offset masks / dictionary optional) */
#define KR_FORMAT_STENCIL 1 /* stencil codes (kr_stencil.h) */
#define KR_FORMAT_DIA 2     /* diagonal-offset values (long masked rows) */
#define KR_FORMAT_DENSE 3   /* dense row block (GEMV) */
#define KR_FORMAT_DIA_WALK 4 /* symmetric diagonal-offset values, row-block walk with the
                              mirrored lower entries in LDS (band <= 256 rows): workgroup
                              g of spmv_grid owns the row blocks [g nb / G, (g+1) nb / G),
                              block g when nb <= G */

/* Halo exchange plan (pure host arithmetic, no device; test hook and the
 * planner kr_system_finalize uses). part[0..nshards] is the global row
 * partition, need_lo[t]..need_hi[t] the global rows shard t's SpMV reads
 * (its own rows included). For shard `me`, writes (peer, first_row, count)
 * triples of the rows it receives (recv_out) and sends (send_out), up to
 * `cap` each; *nrecv / *nsend return the full counts. Replaces the full-vector
 * broadcast + gather of MultiGpu.dot (v3/gpu/common.py:115-122). */
int kr_halo_plan(int nshards, const int64_t* part, const int64_t* need_lo,
                 const int64_t* need_hi, int me, int64_t* recv_out, int* nrecv,
                 int64_t* send_out, int* nsend, int cap);

/* Synthetic right-hand side b[i] = 2*u(seed,i) - 1 (exact in fp64) for this
 * shard's rows, written to b_dev (n_local doubles). */
int kr_fill_rhs(kr_system* sys, int shard, uint64_t seed, double* b_dev);

/* Distributed SpMV of one vector through the halo exchange (test hook):
 * x_dev / y_dev hold the shard's own rows (n_local each). */
int kr_system_spmv(kr_system* sys, const double* const* x_dev, double* const* y_dev);

/* ------------------------------------------------------------------------
 * Solver session: the iteration loops of v3/gpu/<method>.py and
 * v3/gpu/mpi/<method>.py, run natively.
 * ------------------------------------------------------------------------ */
typedef struct {
  int method;      /* KR_METHOD_* */
  int k;           /* k-skip depth (ignored by CG/MrR) */
  double tol;      /* relative residual tolerance */
  int64_t maxiter; /* < 0: n_global (reference default for None,
                      v3/gpu/common.py:35); 0 is honoured (CG / k-skip CG return
                      the initial residual; the MrR family is refused: the
                      reference raises IndexError there) */
  int profile;     /* N > 0: per-kernel HIP-event timing on every N-th outer
                     iteration (1 = all; events cost ~10 us per kernel) */
  int nan_guard;   /* 1: stop at the first NaN/Inf residual entry (reported as
                      not converged, kr_solve_result.diverged = 1). 0 (default):
                      the reference's semantics -- a NaN never passes the tests
                      `res < tol` / `res > pre_res`, so the loop runs on to
                      maxiter (v3/cpu/kskipmrr.py:39-42, v3/common.py:17). */
} kr_solve_params;

typedef struct {
  double time_s;        /* iteration-loop wall time, as info['time'] */
  int64_t iterations;   /* final i (info['nosl'][-1]) */
  int64_t entries;      /* len(info['residual']) */
  int converged;        /* residual < tol reached */
  int final_k;          /* adaptive: final k */
  double final_residual;
  int diverged;         /* nan_guard stopped the loop at a non-finite residual */
} kr_solve_result;

/* Set up vectors, r0 = b - A x0 and ||b||; b_dev[s]/x0_dev[s] hold shard s's
 * own rows (x0 may be NULL for zeros). Starts the timer. */
int kr_solve_begin(kr_system* sys, const kr_solve_params* params,
                   const double* const* b_dev, const double* const* x0_dev);
/* Jacobi preconditioner of the KR_METHOD_PCG .. KR_METHOD_PIPECG sessions
 * begun after this call: d_dev[s] holds shard s's own rows of the diagonal d
 * (M^-1 v = v / d: the `ilu.solve` of v1/threads/pipeline/pcg.py:27,45 and
 * its siblings). The pointers are read at kr_solve_begin (copied into the
 * session); d_dev == NULL restores the identity (d = 1). */
int kr_solve_set_precond(kr_system* sys, const double* const* d_dev);
/* ILU preconditioner for the same family: the reference's `ilu` is a scipy
 * SuperLU (spilu / splu) with A ~ Pr^T L U Pc^T, and `ilu.solve(v)` =
 * Pc U^-1 L^-1 Pr v (v1/threads/pipeline/pcg.py:26,41, gropp.py:25,33,
 * chronopoulos_gear.py:26,46, pipeline.py:26,39). HOST arrays: L and U as
 * CSR rows incl. the diagonal (ascending columns, int64 row pointers, int32
 * columns), perm_r / perm_c as SuperLU gives them (Pr[perm_r[i], i] = 1,
 * Pc[i, perm_c[i]] = 1). Validated and copied at the call (the factors'
 * level schedules are built here); the sweeps run on the device, one
 * workgroup per sweep, levels separated by barriers. Needs a one-shard
 * system (KR_ERR_INVALID otherwise). l_rowptr == NULL clears it; either
 * set_precond call replaces the other's preconditioner. A solve uses the
 * preconditioner set when its kr_solve_begin ran (the factors are shared
 * with the session, the diagonal copied): a later set_precond call, or a
 * clear, takes effect at the next kr_solve_begin. */
int kr_solve_set_precond_ilu(kr_system* sys, int64_t n, const int64_t* l_rowptr,
                             const int32_t* l_col, const double* l_val, const int64_t* u_rowptr,
                             const int32_t* u_col, const double* u_val, const int64_t* perm_r,
                             const int64_t* perm_c);
/* Run up to `max_outer` further outer iterations (CG/MrR: iterations).
 * *done = 1 once converged or maxiter reached. */
int kr_solve_step(kr_system* sys, int64_t max_outer, int* done);
/* Finish: final residual bookkeeping, stop the timer, copy x out. */
int kr_solve_end(kr_system* sys, double* const* x_dev, kr_solve_result* result);
/* Copy the histories (residual, nosl, khistory; khistory may be NULL). */
int kr_solve_history(kr_system* sys, double* residual_host, int64_t* nosl_host,
                     int64_t* khistory_host, int64_t capacity);

/* Per-kernel-class timing (profile != 0): fills up to `cap` records, for the
 * shards on the first shard's device. One launch = one call of the op:
 * total_ms sums the device windows (earliest begin to latest end of those
 * shards' events, whether they share a stream or not), bytes_per_launch is
 * the algorithmic bytes of all of them and `shards` how many
 * shards' launches one call covers (ABI 204). */
typedef struct {
  char name[32];
  int64_t launches;
  double total_ms;
  double bytes_per_launch; /* algorithmic bytes, see DESIGN.md */
  int64_t shards;
} kr_kernel_stat;
int kr_solve_kernel_stats(kr_system* sys, kr_kernel_stat* stats, int cap, int* count);
/* Zero the per-kernel statistics (e.g. after warm-up) and restart the
 * every-N-th sampling (profile = N) with the next outer iteration. */
int kr_solve_kernel_stats_reset(kr_system* sys);

#ifdef __cplusplus
}
#endif
#endif /* KRYLOV_AMD_H */
