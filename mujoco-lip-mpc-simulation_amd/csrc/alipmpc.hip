// alipmpc.hip — MI355X (gfx950) batched ALIP-MPC-CBF footstep planner: HIP kernels + the C ABI of
// include/alipmpc.h.
//
// What it replaces (reference /root/reference):
//   MPCCBF.select_obs / solveMPCCBF / gen_control_test rollout   MPC_LIP_modi.py:90-112, 197-301, 325-338
//   LIP_Prob.objective / gradient / constraints / jacobian       MPC_LIP_modi.py:430-583 (+ helpers 586-655)
//   sig_step variants                                            MPC_LIP_sig_step.py:184-278, 372-496
//   cyipopt.Problem(...).solve(u0)  (IPOPT + MA57)               MPC_LIP_modi.py:274-296
//
// Design (DESIGN.md has the full story):
//   * one NLP instance per 64-lane wavefront, 4 instances per 256-thread workgroup; every
//     synchronisation after the prologue is wave-local, so waves finish independently.
//   * "generator space": the ALIP step-to-step map is affine, so every quantity the NLP touches —
//     the states x_1..x_N and footholds p_0..p_{N-1} — is V = E x0 + G u with a CONSTANT generator
//     matrix G (NG = 8(N+1) rows: block k = [x_k(5), p_k(3)]).  G lives in LDS, shared by the block.
//     Each Jacobian row is <= 4 coefficients on rows of G; each Hessian term is an 8x8 block of one
//     generator block.  Line-search trial points are V + alpha dV: no re-rollout.
//   * KKT matrix K = J^T Sigma J + G^T S G  (n x n, n = 5N <= 30) accumulated with
//     v_mfma_f64_16x16x4_f64 — the A and B fragments of both products are the SAME (row, column)
//     element, so each lane builds its fragment in registers, no LDS staging of J.
//   * K -> LDS transpose -> row-per-lane registers -> Cholesky with readlane broadcasts (compile-time
//     register indices, template on N), forward/back substitution, IPOPT-style inertia correction.
//   * primal-dual interior point, IPOPT's monotone barrier update, fraction-to-boundary rule and filter
//     line search; same algorithm and constants as oracle/np_oracle.py and oracle/alipmpc_oracle.c.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "../../include/alipmpc.h"

// Build partitioning (see the kernel launchers below): ALIP_PART = 0 host code, 1..6 one horizon each.
#ifndef ALIP_PART
#define ALIP_PART_HOST 1
#define ALIP_PART_N(k) 1
#else
#define ALIP_PART_HOST (ALIP_PART == 0)
#define ALIP_PART_N(k) (ALIP_PART == (k))
#endif
// ALIP_PART 7 / 8: the lane solver's fp64 / fp32 kernels (lane_solve.inc)

namespace alip {

constexpr int WAVE = 64;
constexpr int WAVES_PER_BLOCK = 4;
constexpr int MAX_ROWS = 128;        // padded constraint rows per instance (2 per lane)
constexpr int FILTER_CAP = 128;      // 2 filter entries per lane
constexpr int REST_FAIL = 6;         // restoration events with violation > 1e-4 -> status 2


typedef double d4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------------
// kernel parameters (by value)
// ------------------------------------------------------------------------------------------------
struct KP {
    int nc_max, ne_max, rps, m_max, mr4, mo4, modi, max_iter, select_obs, detour;
    int goal_abort;   // cfg.goal_singular == ABORT: an iterate with a planned state on the goal ends with status -13
    int resto_ipopt;  // cfg.restoration == IPOPT (LIP variants): a failed line search enters IPOPT's restoration phase
    uint32_t* redo;          // lane program, cfg.restoration = IPOPT: [0] = count, then the instances whose line search
                             // failed (their solve is handed to the fp64 wave program, which has the restoration phase)
    const uint32_t* bcount;  // nullable: the work-queue form solves instances order[k] for k < min(B, *bcount)
    double tol, acc_tol, q, p, r, gm1, s, detect_r2, leg2, bvx_lo, bvx_hi, bvy_lo, bvy_hi, dth, mu_init, dt, dd_t;
    const double* G;   // NG x NCP
    const double* E;   // NG x 5
    const double* Gu;  // NG x NCPU : u-parametrisation V = Eu x0 + Gu u (warm start u0 -> p0)
    const double* Eu;  // NG x 5
    long long B;
    const double* x0;
    const double* goal;
    const int8_t* leg;
    const double* cir;
    const int32_t* nc;
    const double* elp;
    const int32_t* ne;
    const double* u0;
    const double* last_u;   // DD: previous control (B x 2)
    const uint8_t* active;  // nullable: instances with active[b] == 0 are skipped (closed-loop rollouts)
    uint32_t* queue;        // nullable: work-queue counters of a persistent solve launch (solve_kernel)
    const int32_t* order;   // nullable: launch order of the wave program (wave / queue slot k solves instance
                            // order[k]; the closed loop puts last tick's long instances first)
    int ckpt_it;            // split launch, phase 1 (> 0): an instance still running at this iteration saves its
                            // loop state to a record and stops (solve_kernel, one wave per instance)
    int resume;             // split launch, phase 2: wave k resumes the instance of record k
    int ckpt_tr;            // split launch, phase 1 (> 0, with team > 0): an instance whose line search has run this
                            // many trials also stops (before ckpt_it) and gets a TEAM record
    int team;               // split launch (team-capable build): phase 1 — team records on (ckpt_tr); phase 2 — team
                            // workgroups ahead of the single ones (each runs one team record on its 4 waves in lockstep,
                            // consecutive line-search trials per round)
    double* ckpt;           // split launch: per-record loop state (ckpt_doubles(mo4) each)
    uint32_t* cont;         // split launch counters (CONT_*): single / team records, then the instance of record k
                            // (singles from k = 0 up, team record j at k = B - 1 - j)
    // solve outputs
    double* u_out;
    double* foot_out;
    double* x_pred;
    int32_t* status;
    int32_t* iters;
    // eval outputs
    double* f_out;
    double* grad_out;
    double* c_out;
    double* J_out;
    double* cl_out;
    double* cu_out;
    double* goal_eff_out;
    int8_t* active_out;
    // lane-solver constants (lane_solve.inc, LK_* slots) in device memory, fp64 and an fp32 copy
    const double* lkd;
    const float* lkfd;
};

constexpr int KP_DOUBLES = (int)((sizeof(KP) + 15) / 16 * 2);
constexpr int FAIL_GOAL = 1 << 16;   // solve_kernel's fail_it tag of a cfg.goal_singular = ABORT exit
// split-launch record of one instance: per lane and row group the row state (slack, multipliers, inverse slack
// distances, value, transcendentals, the 4 generator values), the filter entries (2 x 2) and the generator value
// V[lane]; then 16 uniform values
// Split record layout (r6: live state only): CKPT_ROW row vectors of the instance's mo4 rows
// (value i of row r at i * mo4 + r), the filter (entry j at CK_FILT + j for theta, + 128 for phi; only the nf live
// entries are written and read), the iterate V (NG <= 56 lanes) and 13 scalars.  cfg2 (mo4 = 40): 6.5 KB per record,
// ~4.7 KB written and read per cut instance (r5: 8.8 KB, all 64 lanes of every vector).
constexpr int CKPT_ROW = 12;
__host__ __device__ constexpr int ck_filt(int mo4) { return CKPT_ROW * mo4; }
__host__ __device__ constexpr int ck_vme(int mo4) { return CKPT_ROW * mo4 + 4 * WAVE; }
__host__ __device__ constexpr int ck_scal(int mo4) { return CKPT_ROW * mo4 + 4 * WAVE + 56; }
__host__ __device__ constexpr int ckpt_doubles(int mo4) { return CKPT_ROW * mo4 + 4 * WAVE + 56 + 16; }
#ifndef ALIP_SPLIT_IT
#define ALIP_SPLIT_IT 14   // (r5 sweep on cfg2: 12 / 13 / 14 / 15 / 16 / 18 / 20 = 0.58 / 0.59 / 0.537 / 0.55 / 0.543 / 0.545 / 0.55 ms)
#endif
constexpr int SPLIT_IT_DEFAULT = ALIP_SPLIT_IT;   // phase-1 iteration cap of the split launch (launch_solve)
// with IPOPT's restoration phase (cfg.restoration, r6: a failed search in phase 1 is cut there, so the restoration
// instances reach phase 2 earlier; sweep on cfg2: 12 / 13 / 14 / 15 / 16 / 17 / 18 / 20 = 0.636 / 0.630 / 0.646 /
// 0.653 / 0.613 / 0.626 / 0.641 / 0.650 ms)
constexpr int SPLIT_IT_DEFAULT_RESTO = 16;
constexpr int SPLIT_TR_DEFAULT = 0;               // phase-1 trial cut of a cold solve (0 = off: no team records)
constexpr int CL_SPLIT_IT_DEFAULT = 20;           // the closed loop's per-tick solves: phase-1 cap (r5: 16 / 18 / 20 / 22 /
                                                   // 24 = 23.7 / 22.95 / 22.7 / 22.8 / 23.6 ms per loop)
constexpr int CL_SPLIT_TR_DEFAULT = 40;           // and trial cut
constexpr int CL_GROUPS_DEFAULT = 2;              // closed loop: episode groups on streams of their own (4: host-bound)
static int env_groups()
{
    const char* t = std::getenv("ALIPMPC_CL_GROUPS");
    return t ? std::max(1, std::atoi(t)) : CL_GROUPS_DEFAULT;
}
// split-launch counters (KP.cont): single records, team records, then the B instance ids of records (index k)
constexpr int CONT_SINGLE = 0, CONT_TEAM = 1;
__host__ __device__ constexpr long long cont_hdr(long long) { return 2; }
constexpr long long TEAM_CAP = 128;   // team workgroups of a phase-2 launch (team records beyond run one wave each)
// waves of a team-capable workgroup = members of a team, each testing one of that many consecutive line-search trials
// per round.  r5 measured 8 against 4: the closed loop 33.8 vs 31.1 ms — every member also
// runs the whole direction computation, and 8 of them share their SIMDs with the other episode group's phase 1
// (profiles/r5/closed_loop); 4 kept
#ifndef ALIP_TEAM_WAVES
#define ALIP_TEAM_WAVES 4
#endif
constexpr int TEAM_WAVES = ALIP_TEAM_WAVES;
#ifndef ALIP_GJ_REGS
#define ALIP_GJ_REGS 1
#endif
#ifndef ALIP_GJ_MAX_N   // largest KKT size solved by Gauss-Jordan (register rows); larger n: register Cholesky
#define ALIP_GJ_MAX_N 15  // (cfg3, n = 15: 16.14 -> 15.51 ms per launch against the Cholesky)
#endif
constexpr int ST_CKPT = 3;   // internal status of an instance whose loop state went to a split-launch record
constexpr int ST_RESTO = 4;  // internal: a failed line search hands the point to IPOPT's restoration phase
// record slots are doubles; an fp32 kernel's values are stored as their bit patterns (no conversion)
__device__ __forceinline__ double ck_put(double v) { return v; }
__device__ __forceinline__ double ck_put(float v) { return __longlong_as_double((long long)__float_as_uint(v)); }
template <class R>
__device__ __forceinline__ R ck_get(double d);
template <>
__device__ __forceinline__ double ck_get<double>(double d) { return d; }
template <>
__device__ __forceinline__ float ck_get<float>(double d) { return __uint_as_float((unsigned)__double_as_longlong(d)); }

// R_FEN is the reference's f_en row (eval); in the solve layout (modi) it is the smooth half
// vbx + s dth <= bvx_hi and R_FENM the other half vbx - s dth <= bvx_hi (see row_bounds)
enum RowType { R_VBX = 0, R_VBY, R_CIR, R_ELP, R_LEG, R_DTH, R_FEN, R_FENM, R_NONE, R_OBJ };

// ---- diagnostic phase timers (compiled only with -DALIP_STAMPS; never in the product build)
#ifdef ALIP_STAMPS
constexpr int NSTAMP = 26;   // 0-9 solve_one's sections, 10-21 resto_wave's, 22 / 23 restoration calls / iterations,
                             // 24 solve_one's re-evaluation after a restoration, 25 the restoration call as solve_one
                             // sees it (hand-over to LDS + resto_wave)
__device__ unsigned long long g_stamps[NSTAMP];
#define STAMP_DECL unsigned long long st_acc[NSTAMP] = {}; unsigned long long st_t = __builtin_amdgcn_s_memtime();
#define STAMP(i)                                                              \
    do {                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                    \
        unsigned long long t_ = __builtin_amdgcn_s_memtime();                 \
        st_acc[i] += t_ - st_t;                                               \
        st_t = t_;                                                            \
        __builtin_amdgcn_sched_barrier(0);                                    \
    } while (0)
#define STAMP_FLUSH                                                           \
    do {                                                                      \
        if (lane_id() == 0)                                                   \
            for (int i_ = 0; i_ < NSTAMP; ++i_) atomicAdd(&g_stamps[i_], st_acc[i_]); \
    } while (0)
#define RSTAMP_DECL unsigned long long rs_acc[12] = {}; unsigned long long rs_t = __builtin_amdgcn_s_memtime();
#define RSTAMP(i)                                                             \
    do {                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                    \
        unsigned long long t_ = __builtin_amdgcn_s_memtime();                 \
        rs_acc[i] += t_ - rs_t;                                               \
        rs_t = t_;                                                            \
        __builtin_amdgcn_sched_barrier(0);                                    \
    } while (0)
#define RSTAMP_FLUSH(nit)                                                     \
    do {                                                                      \
        if (lane_id() == 0) {                                                 \
            for (int i_ = 0; i_ < 12; ++i_) atomicAdd(&g_stamps[10 + i_], rs_acc[i_]); \
            atomicAdd(&g_stamps[22], 1ull);                                   \
            atomicAdd(&g_stamps[23], (unsigned long long)(nit));              \
        }                                                                     \
    } while (0)
#else
#define STAMP_DECL
#define STAMP(i) do {} while (0)
#define STAMP_FLUSH do {} while (0)
#define RSTAMP_DECL
#define RSTAMP(i) do {} while (0)
#define RSTAMP_FLUSH(nit) do {} while (0)
#endif

// ---- diagnostic per-instance record of the wave program (compiled only with -DALIP_WSTAMP; never in the product
// build): [start, end] of the instance on the constant 100 MHz clock and the shader clock, HW_ID / XCC_ID of the wave,
// iterations, line-search trials, restorations.  Slot = g_wstamp_base + instance (the closed loop sets the base per
// tick), 8 values per slot, written by lanes 0..7 (vector stores).  tools/cl_wstamps.py reads it.
#ifdef ALIP_WSTAMP
constexpr long long WSTAMP_CAP = 48 * 4096;
__device__ unsigned long long g_wstamp[WSTAMP_CAP * 8];
__device__ long long g_wstamp_base;
#define WSTAMP_DECL                                                                        \
    const unsigned long long ws_t0 = __builtin_amdgcn_s_memrealtime();                    \
    const unsigned long long ws_c0 = __builtin_amdgcn_s_memtime();                        \
    unsigned ws_trials = 0;
#define WSTAMP_TRIAL ++ws_trials
#define WSTAMP_WRITE(b, it, nrest)                                                         \
    do {                                                                                   \
        const unsigned long long t1_ = __builtin_amdgcn_s_memrealtime();                   \
        const unsigned long long c1_ = __builtin_amdgcn_s_memtime();                       \
        const unsigned hw_ = __builtin_amdgcn_s_getreg(4 | (31 << 11));                   \
        const unsigned xcc_ = __builtin_amdgcn_s_getreg(20 | (15 << 11));                 \
        const long long slot_ = g_wstamp_base + (b);                                       \
        const int l_ = lane_id();                                                          \
        unsigned long long v_ = l_ == 0 ? ws_t0 : l_ == 1 ? t1_ : l_ == 2 ? ws_c0 : l_ == 3 ? c1_ \
                              : l_ == 4 ? ((unsigned long long)xcc_ << 32 | hw_)                \
                              : l_ == 5 ? (unsigned long long)(it) : l_ == 6 ? (unsigned long long)ws_trials \
                              : (unsigned long long)(nrest);                               \
        if (slot_ >= 0 && slot_ < WSTAMP_CAP && l_ < 8) g_wstamp[slot_ * 8 + l_] = v_;     \
    } while (0)
#else
#define WSTAMP_DECL
#define WSTAMP_TRIAL do {} while (0)
#define WSTAMP_WRITE(b, it, nrest) do {} while (0)
#endif

template <int N>
struct Dim {
    static constexpr int n = 3 * N;     // decision = footholds p_0..p_{N-1} (see build_tables)
    static constexpr int NT = (n + 15) / 16;
    static constexpr int NCP = 16 * NT;
    static constexpr int nu = 5 * N;    // the reference's decision u (eval / warm start)
    static constexpr int NTU = (nu + 15) / 16;
    static constexpr int NCPU = 16 * NTU;
    static constexpr int NG = 8 * (N + 1);
    static constexpr int KLD = NCP + 1;
};

// ------------------------------------------------------------------------------------------------
// wave-level helpers
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & (WAVE - 1); }

__device__ __forceinline__ void wave_sync()
{
    // LDS hand-off between lanes of ONE wave.  A wavefront's DS instructions execute in order, so no
    // s_waitcnt / s_barrier is needed — only a compiler barrier that keeps the accesses in program order.
    // (The 4 waves of a workgroup run different instances and never synchronise with each other.)
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// wave-uniform int (SGPR)
__device__ __forceinline__ int rfl(int x) { return __builtin_amdgcn_readfirstlane(x); }
// Opaque copy of a per-lane value: addresses derived from it are recomputed after this point instead of
// being hoisted out of the interior-point loop (dozens of hoisted LDS addresses otherwise spill).
#define RELAUNDER(x) asm volatile("" : "+v"(x))

// a wave-uniform double: pins it to an SGPR pair (long-lived uniform values otherwise occupy VGPRs)
__device__ __forceinline__ double uni(double v)
{
    const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
    const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double bcast(double v, int src)
{
    int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
    int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
    return __hiloint2double(hi, lo);
}

// ---- cross-lane exchange without LDS: DPP within 16-lane rows, permlane swaps across rows
template <int CTRL>
__device__ __forceinline__ double dpp(double v)
{
    int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
// returns (v[l], v[l ^ 16]) / (v[l], v[l ^ 32]) as the symmetric pair (a, b)
__device__ __forceinline__ void swap16(double v, double& a, double& b)
{
    auto lo = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(v), (unsigned)__double2loint(v), false, false);
    auto hi = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(v), (unsigned)__double2hiint(v), false, false);
    a = __hiloint2double((int)hi[0], (int)lo[0]);
    b = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ void swap32(double v, double& a, double& b)
{
    auto lo = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(v), (unsigned)__double2loint(v), false, false);
    auto hi = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(v), (unsigned)__double2hiint(v), false, false);
    a = __hiloint2double((int)hi[0], (int)lo[0]);
    b = __hiloint2double((int)hi[1], (int)lo[1]);
}

// fp32 counterparts (the solve kernel is templated on its arithmetic type R, cfg.precision)
__device__ __forceinline__ float uni(float v)
{
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ __forceinline__ float bcast(float v, int src)
{
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), src));
}
template <int CTRL>
__device__ __forceinline__ float dpp(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ void swap16(float v, float& a, float& b)
{
    auto x = __builtin_amdgcn_permlane16_swap((unsigned)__float_as_int(v), (unsigned)__float_as_int(v), false, false);
    a = __int_as_float((int)x[0]);
    b = __int_as_float((int)x[1]);
}
__device__ __forceinline__ void swap32(float v, float& a, float& b)
{
    auto x = __builtin_amdgcn_permlane32_swap((unsigned)__float_as_int(v), (unsigned)__float_as_int(v), false, false);
    a = __int_as_float((int)x[0]);
    b = __int_as_float((int)x[1]);
}

struct OpAdd {
    template <class T>
    __device__ T operator()(T a, T b) const { return a + b; }
};
struct OpMax {
    template <class T>
    __device__ T operator()(T a, T b) const { return fmax(a, b); }
};
struct OpMin {
    template <class T>
    __device__ T operator()(T a, T b) const { return fmin(a, b); }
};

// butterfly over all 64 lanes; every lane receives the result.
//   quad_perm [1,0,3,2] (l^1), quad_perm [2,3,0,1] (l^2), row_half_mirror (quads of a half-row),
//   row_mirror (half-rows), permlane16_swap (l^16), permlane32_swap (l^32)
template <class T, class Op>
__device__ __forceinline__ T wreduce(T v, Op op)
{
    v = op(v, dpp<0xB1>(v));
    v = op(v, dpp<0x4E>(v));
    v = op(v, dpp<0x141>(v));
    v = op(v, dpp<0x140>(v));
    T a, b;
    swap16(v, a, b);
    v = op(a, b);
    swap32(v, a, b);
    return uni(op(a, b));
}
template <class T>
__device__ __forceinline__ T wsum(T v) { return wreduce(v, OpAdd()); }
template <class T>
__device__ __forceinline__ T wmax(T v) { return wreduce(v, OpMax()); }
template <class T>
__device__ __forceinline__ T wmin(T v) { return wreduce(v, OpMin()); }
template <class T>
__device__ __forceinline__ void wsum2(T& a, T& b)
{
    a = wsum(a);
    b = wsum(b);
}
// sum over the 4 lane groups (lanes c, c+16, c+32, c+48)
template <class T>
__device__ __forceinline__ T gsum(T v)
{
    T a, b;
    swap16(v, a, b);
    v = a + b;
    swap32(v, a, b);
    return a + b;
}

// ---- type-generic scalar pieces of the solve kernel (R = double | float)

// 4 consecutive LDS values (16-byte aligned) as b128 accesses
__device__ __forceinline__ void ld4(const double* p, double& a, double& b, double& c, double& d)
{
    const double2* q = reinterpret_cast<const double2*>(p);
    const double2 x = q[0], y = q[1];
    a = x.x; b = x.y; c = y.x; d = y.y;
}
__device__ __forceinline__ void ld4(const float* p, float& a, float& b, float& c, float& d)
{
    const float4 x = *reinterpret_cast<const float4*>(p);
    a = x.x; b = x.y; c = x.z; d = x.w;
}
__device__ __forceinline__ void st4(double* p, double a, double b, double c, double d)
{
    double2* q = reinterpret_cast<double2*>(p);
    q[0] = make_double2(a, b);
    q[1] = make_double2(c, d);
}
__device__ __forceinline__ void st4(float* p, float a, float b, float c, float d)
{
    *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
}

// 16x16x4 MFMA with one operand element per lane (A[l&15][l>>4], B[l>>4][l&15]).  C/D layout: f64
// row = (l>>4) + 4 i, f32 row = 4 (l>>4) + i (cdna_hip_programming.md §3), col = l & 15.
typedef float f4 __attribute__((ext_vector_type(4)));
template <class R>
struct Mfma;
template <>
struct Mfma<double> {
    typedef d4 acc;
    __device__ static __forceinline__ d4 run(double a, double b, d4 c)
    {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    __device__ static __forceinline__ int row(int g4, int i) { return g4 + 4 * i; }
};
template <>
struct Mfma<float> {
    typedef f4 acc;
    __device__ static __forceinline__ f4 run(float a, float b, f4 c)
    {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    __device__ static __forceinline__ int row(int g4, int i) { return 4 * g4 + i; }
};

// generator row indices
__device__ __forceinline__ int gx(int k, int c) { return 8 * k + c; }       // state x_k comp c
__device__ __forceinline__ int gp(int k, int c) { return 8 * k + 5 + c; }   // foothold p_k comp c

// ------------------------------------------------------------------------------------------------
// row decode + evaluation.  Returns the row type; c = value; coef/gen = Jacobian in generator form.
// ------------------------------------------------------------------------------------------------
struct RowInfo {
    int type, k, slot;
};

__device__ __forceinline__ RowInfo decode_row(const KP& P, int r, int nc_sel, int ne_sel)
{
    RowInfo ri;
    ri.k = r / P.rps;
    int l = r - ri.k * P.rps;
    ri.slot = 0;
    if (r >= P.m_max) {
        ri.type = R_NONE;
    } else if (l == 0) {
        ri.type = R_VBX;
    } else if (l == 1) {
        ri.type = R_VBY;
    } else if (l < 2 + P.nc_max) {
        ri.slot = l - 2;
        ri.type = ri.slot < nc_sel ? R_CIR : R_NONE;
    } else if (l < 2 + P.nc_max + P.ne_max) {
        ri.slot = l - 2 - P.nc_max;
        ri.type = ri.slot < ne_sel ? R_ELP : R_NONE;
    } else if (l == 2 + P.nc_max + P.ne_max) {
        ri.type = R_LEG;
    } else if (l == 3 + P.nc_max + P.ne_max) {
        ri.type = R_DTH;
    } else if (l == 4 + P.nc_max + P.ne_max) {
        ri.type = R_FEN;
    } else {
        ri.type = R_FENM;   // solve layout only
    }
    return ri;
}

// split (solve layout, modi): f_en = vbx + s|dth| in [bvx_lo, bvx_hi] becomes vbx +- s dth <= bvx_hi — the
// same feasible set (|x| <= c <=> +-x <= c; the lower bound is implied by the vbx row since s > 0), but
// smooth, so Newton steps are not trapped at the kink dth = 0.
template <class R>
__device__ __forceinline__ void row_bounds(const KP& P, const RowInfo& ri, int leg, R& cl, R& cu, bool split = false)
{
    switch (ri.type) {
    case R_VBX:
        cl = P.bvx_lo;
        cu = P.bvx_hi;
        break;
    case R_FEN:
    case R_FENM:
        cl = split ? -INFINITY : P.bvx_lo;
        cu = P.bvx_hi;
        break;
    case R_VBY: {
        bool pos = (leg > 0) == ((ri.k & 1) == 0);
        cl = pos ? P.bvy_lo : -P.bvy_hi;
        cu = pos ? P.bvy_hi : -P.bvy_lo;
        break;
    }
    case R_CIR:
    case R_ELP:
        cl = R(0);
        cu = INFINITY;
        break;
    case R_LEG:
        cl = R(0);
        cu = P.leg2;
        break;
    case R_DTH:
        cl = R(-P.dth);
        cu = P.dth;
        break;
    default:
        cl = -INFINITY;
        cu = INFINITY;
    }
}

__device__ __forceinline__ void sabs(double x, double eps, double& v, double& d1, double& d2)
{
    if (eps == 0.0) {
        v = fabs(x);
        d1 = x == 0.0 ? 0.0 : copysign(1.0, x);
        d2 = 0.0;
    } else {
        double r = sqrt(x * x + eps * eps);
        v = r;
        d1 = x / r;
        d2 = eps * eps / (r * r * r);
    }
}

template <int N, bool JAC>
__device__ __forceinline__ double row_eval(const KP& P, const RowInfo& ri, const double* V, const double* CT, const double* ST,
                           const double* obs, double eps, double* coef, int* gen)
{
    const int k = ri.k;
    double c = 0.0;
    if (JAC) {
        coef[0] = coef[1] = coef[2] = coef[3] = 0.0;
        gen[0] = gen[1] = gen[2] = gen[3] = 0;
    }
    switch (ri.type) {
    case R_VBX:
    case R_VBY:
    case R_FEN: {
        double ct = CT[k + 1], st = ST[k + 1];
        double vx = V[gx(k + 1, 2)], vy = V[gx(k + 1, 3)];
        double vbx = ct * vx + st * vy;
        if (ri.type == R_VBY) {
            c = -st * vx + ct * vy;
            if (JAC) {
                coef[0] = -st; coef[1] = ct; coef[2] = -ct * vx - st * vy;
                gen[0] = gx(k + 1, 2); gen[1] = gx(k + 1, 3); gen[2] = gx(k + 1, 4);
            }
        } else {
            c = vbx;
            if (JAC) {
                coef[0] = ct; coef[1] = st; coef[2] = -st * vx + ct * vy;
                gen[0] = gx(k + 1, 2); gen[1] = gx(k + 1, 3); gen[2] = gx(k + 1, 4);
            }
            if (ri.type == R_FEN) {
                double a, d1, d2;
                sabs(V[gp(k, 2)], eps, a, d1, d2);
                c += P.s * a;
                if (JAC) {
                    coef[3] = P.s * d1;
                    gen[3] = gp(k, 2);
                }
            }
        }
        break;
    }
    case R_CIR: {
        const double* o = obs + 3 * ri.slot;
        double x1 = V[gx(k + 1, 0)] - o[0], y1 = V[gx(k + 1, 1)] - o[1];
        double x0 = V[gx(k, 0)] - o[0], y0 = V[gx(k, 1)] - o[1];
        double rr = o[2] * o[2];
        c = (x1 * x1 + y1 * y1 - rr) + P.gm1 * (x0 * x0 + y0 * y0 - rr);
        if (JAC) {
            coef[0] = 2 * x1; coef[1] = 2 * y1; coef[2] = P.gm1 * 2 * x0; coef[3] = P.gm1 * 2 * y0;
            gen[0] = gx(k + 1, 0); gen[1] = gx(k + 1, 1); gen[2] = gx(k, 0); gen[3] = gx(k, 1);
        }
        break;
    }
    case R_ELP: {
        const double* o = obs + 3 * P.nc_max + 5 * ri.slot;
        const double* qq = obs + 3 * P.nc_max + 5 * P.ne_max;
        double qa = qq[ri.slot], qb = qq[P.ne_max + ri.slot], qc = qq[2 * P.ne_max + ri.slot], ek = qq[3 * P.ne_max + ri.slot];
        double x1 = V[gx(k + 1, 0)] - o[0], y1 = V[gx(k + 1, 1)] - o[1];
        double x0 = V[gx(k, 0)] - o[0], y0 = V[gx(k, 1)] - o[1];
        c = (qa * x1 * x1 + qb * x1 * y1 + qc * y1 * y1 - ek) + P.gm1 * (qa * x0 * x0 + qb * x0 * y0 + qc * y0 * y0 - ek);
        if (JAC) {
            coef[0] = 2 * qa * x1 + qb * y1; coef[1] = 2 * qc * y1 + qb * x1;
            coef[2] = P.gm1 * (2 * qa * x0 + qb * y0); coef[3] = P.gm1 * (2 * qc * y0 + qb * x0);
            gen[0] = gx(k + 1, 0); gen[1] = gx(k + 1, 1); gen[2] = gx(k, 0); gen[3] = gx(k, 1);
        }
        break;
    }
    case R_LEG: {
        double ex = V[gx(k, 0)] - V[gp(k, 0)], ey = V[gx(k, 1)] - V[gp(k, 1)];
        c = ex * ex + ey * ey;
        if (JAC) {
            coef[0] = 2 * ex; coef[1] = 2 * ey; coef[2] = -2 * ex; coef[3] = -2 * ey;
            gen[0] = gx(k, 0); gen[1] = gx(k, 1); gen[2] = gp(k, 0); gen[3] = gp(k, 1);
        }
        break;
    }
    case R_DTH:
        c = V[gp(k, 2)];
        if (JAC) {
            coef[0] = 1.0;
            gen[0] = gp(k, 2);
        }
        break;
    default:
        break;
    }
    return c;
}

// ------------------------------------------------------------------------------------------------
// solve-instance prologue: load inputs, select_obs, detour goal, ellipse forms, V = E x0 + G p0.
// Computed in fp64 for either workspace type (the discrete select/detour decisions do not depend on
// cfg.precision); results are stored into the workspace's type.
// ------------------------------------------------------------------------------------------------
// 1/sqrt(d) and 1/x to ~1 ulp: hardware estimate + two Newton steps (a few FMAs instead of the
// ~15-instruction IEEE sqrt / div sequences on the Cholesky critical path)
// binary exponent of a normal nonzero value (the trial count of a line search from a = ap 2^-j)
__device__ __forceinline__ int fexp2(double x) { return __builtin_amdgcn_frexp_exp(x); }
__device__ __forceinline__ int fexp2(float x) { return __builtin_amdgcn_frexp_expf(x); }

__device__ __forceinline__ double rsqrt_nr(double d)
{
    double y = __builtin_amdgcn_rsq(d);
    const double h = 0.5 * d;
    y = y * fma(-h * y, y, 1.5);
    y = y * fma(-h * y, y, 1.5);
    return y;
}
__device__ __forceinline__ double rcp_nr(double x)
{
    double y = __builtin_amdgcn_rcp(x);
    double e = fma(-x, y, 1.0);
    y = fma(y, e, y);
    e = fma(-x, y, 1.0);
    return fma(y, e, y);
}
// fp32: the hardware estimates are ~1 ulp already; one Newton step makes them correctly rounded-ish
__device__ __forceinline__ float rsqrt_nr(float d)
{
    float y = __builtin_amdgcn_rsqf(d);
    return y * fmaf(-0.5f * d * y, y, 1.5f);
}
__device__ __forceinline__ float rcp_nr(float x)
{
    float y = __builtin_amdgcn_rcpf(x);
    return fmaf(y, fmaf(-x, y, 1.0f), y);
}

#include "fastmath.inc"

template <int N, class WT>
__device__ void prologue(const KP& P, const WT& w, const typename WT::real* G, const double* E,
                         long long b, double& gxg, double& gyg, int& legv, double& uj)
{
    using D = Dim<N>;
    const int lane = lane_id();
    const double* x0 = P.x0 + 5 * b;
    legv = P.leg[b];
    const int ncr = P.nc[b];
    const int ner = P.ne ? P.ne[b] : 0;
    double x0v0 = x0[0], x0v1 = x0[1];
    double g0 = P.goal[2 * b], g1 = P.goal[2 * b + 1];
    // select_obs (MPC_LIP_modi.py:325-338): keep order, compact into the first slots
    {
        bool valid = lane < ncr && lane < P.nc_max;
        double c0 = 0, c1 = 0, c2 = 0;
        if (valid) {
            const double* c = P.cir + ((size_t)b * P.nc_max + lane) * 3;
            c0 = c[0]; c1 = c[1]; c2 = c[2];
        }
        double d = (x0v0 - c0) * (x0v0 - c0) + (x0v1 - c1) * (x0v1 - c1) - c2 * c2;
        bool keep = valid && (!P.select_obs || d <= P.detect_r2);
        unsigned long long m = __ballot(keep);
        int pos = __builtin_popcountll(m & ((1ull << lane) - 1ull));
        if (keep) {
            w.obs[3 * pos + 0] = c0;
            w.obs[3 * pos + 1] = c1;
            w.obs[3 * pos + 2] = c2;
        }
        if (lane == 0) w.nsel[0] = __builtin_popcountll(m);
    }
    if (P.ne_max > 0) {
        bool valid = lane < ner && lane < P.ne_max;
        double e[5] = {0, 0, 0, 0, 0};
        if (valid) {
            const double* ep = P.elp + ((size_t)b * P.ne_max + lane) * 5;
            for (int i = 0; i < 5; ++i) e[i] = ep[i];
        }
        double rmax = e[2] > e[3] ? e[2] : e[3];
        double d = (x0v0 - e[0]) * (x0v0 - e[0]) + (x0v1 - e[1]) * (x0v1 - e[1]) - rmax * rmax;
        bool keep = valid && (!P.select_obs || d <= P.detect_r2);
        unsigned long long m = __ballot(keep);
        int pos = __builtin_popcountll(m & ((1ull << lane) - 1ull));
        if (keep) {
            auto* o = w.obs + 3 * P.nc_max + 5 * pos;
            for (int i = 0; i < 5; ++i) o[i] = e[i];
            double ce, se;
            sincos(e[4], &se, &ce);
            auto* qq = w.obs + 3 * P.nc_max + 5 * P.ne_max;
            qq[pos] = (e[3] * ce) * (e[3] * ce) + (e[2] * se) * (e[2] * se);
            qq[P.ne_max + pos] = 2 * ce * se * (e[3] * e[3] - e[2] * e[2]);
            qq[2 * P.ne_max + pos] = (e[3] * se) * (e[3] * se) + (e[2] * ce) * (e[2] * ce);
            qq[3 * P.ne_max + pos] = (e[3] * e[2]) * (e[3] * e[2]);
        }
        if (lane == 0) w.nsel[1] = __builtin_popcountll(m);
    } else if (lane == 0) {
        w.nsel[1] = 0;
    }
    wave_sync();
    // detour goal (MPC_LIP_modi.py:247-271): first selected circle that triggers
    gxg = g0;
    gyg = g1;
    if (P.detour) {
        const int ncs = w.nsel[0];
        bool fire = false;
        double nx = 0, ny = 0;
        if (lane < ncs) {
            const auto* c = w.obs + 3 * lane;
            double cen = fma(x0v0 - c[0], x0v0 - c[0], (x0v1 - c[1]) * (x0v1 - c[1]));
            double gd = fma(x0v0 - g0, x0v0 - g0, (x0v1 - g1) * (x0v1 - g1));
            if (cen < gd && cen < 9 * c[2] * c[2]) {
                double th = latan2(g1 - x0v1, g0 - x0v0);   // (the lane program's and the eval hook's functions)
                double al = latan2(c[1] - x0v1, c[0] - x0v0);
                double dd = th - al;
                if (dd < 0 && fabs(dd) > M_PI)
                    dd += 2 * M_PI;
                else if (dd > 0 && fabs(dd) > M_PI)
                    dd -= 2 * M_PI;
                if (fabs(dd) < M_PI / 12) {
                    fire = true;
                    double na = dd < 0 ? th - M_PI / 12 : th + M_PI / 12;
                    double rr = sqrt(gd);
                    double sn, cs;
                    lsincos(na, &sn, &cs);
                    nx = fma(rr, cs, x0v0);   // (explicit fma: every kernel's detour goal rounds alike)
                    ny = fma(rr, sn, x0v1);
                }
            }
        }
        unsigned long long m = __ballot(fire);
        if (m) {
            int first = __builtin_ctzll(m);
            gxg = bcast(nx, first);
            gyg = bcast(ny, first);
        }
    }
    // warm start p0 = rows p_k of (Eu x0 + Gu u0) — the rollout of the reference's u0 — then
    // V = E x0 + G p0 with the foothold tables.
    constexpr int nu = D::nu;
    const double u0v = lane < nu ? P.u0[(size_t)b * nu + lane] : 0.0;
    const double xv = lane < 5 ? x0[lane] : 0.0;
    double xb[5];
#pragma unroll
    for (int c = 0; c < 5; ++c) xb[c] = bcast(xv, c);
    if (lane < nu) w.Vt[lane] = u0v;
    wave_sync();
    if (lane < D::n) {
        const int t = 8 * (lane / 3) + 5 + lane % 3;      // generator row of p_k[c]
        double v = 0.0;
#pragma unroll
        for (int c = 0; c < 5; ++c) v += P.Eu[t * 5 + c] * xb[c];
        const double* gr = P.Gu + (size_t)t * D::NCPU;
        for (int j = 0; j < nu; ++j) v += gr[j] * w.Vt[j];
        uj = v;
    }
    wave_sync();
    if (lane < D::n) w.Vt[lane] = uj;
    wave_sync();
    for (int t = lane; t < D::NG; t += WAVE) {
        double v = 0.0;
#pragma unroll
        for (int c = 0; c < 5; ++c) v += E[t * 5 + c] * xb[c];
        const auto* gr = G + t * D::NCP;
#pragma unroll
        for (int j = 0; j < D::n; ++j) v += gr[j] * w.Vt[j];
        w.V[t] = v;
    }
    wave_sync();
}


// ------------------------------------------------------------------------------------------------
// register Cholesky: lane i (< n) holds row i of the (regularised) KKT matrix in a[0..n-1].
// Right-looking; column j is broadcast with readlane (uniform lane index, compile-time register).
// On success lane i holds row i of L in a[0..i] and idg[j] = 1 / L[j][j] (uniform).
// ------------------------------------------------------------------------------------------------
template <int n, class R>
__device__ __forceinline__ bool chol_rows(R (&a)[n], R& myidg, int lane)
{
#pragma unroll
    for (int j = 0; j < n; ++j) {
        const R d = bcast(a[j], j);
        if (!(d > R(0))) return false;   // wave-uniform
        const R inv = rsqrt_nr(d);
        myidg = lane == j ? inv : myidg;
        const R lij = a[j] * inv;
        a[j] = lane == j ? d * inv : lij;
#pragma unroll
        for (int k = j + 1; k < n; ++k) a[k] -= lij * bcast(lij, k);
    }
    return true;
}

// ------------------------------------------------------------------------------------------------
// Gauss-Jordan solve of the (regularised) KKT system in LDS: M = [K | rhs] (n x (n+1), row stride LD), one
// wave, element e = lane + 64 q owns M[e / (n+1)][e % (n+1)].  Step p: pivot d = M[p][p] (an LDS broadcast;
// for a symmetric matrix the pivots are the D of K = L D L^T, so "all pivots > 0" is exactly the Cholesky
// positive-definiteness test the inertia correction needs), row p /= d, every other row -= M[i][p] row p.
// All reads of a step precede its writes in program order and a wave's DS operations execute in order, so
// no barrier is needed.  n steps of ~3 LDS reads + 1 write per element group replace the register
// Cholesky's O(n^2) readlane broadcasts and the two sequential triangular sweeps.  On success column n
// holds the solution.
// ------------------------------------------------------------------------------------------------
template <int n, int LD, class R>
__device__ __forceinline__ bool gj_lds(R* M, int lane)
{
    constexpr int NE = n * (n + 1), Q = (NE + WAVE - 1) / WAVE;
    // lanes past the last element work on the padding element M[n][n] (row n is not part of the system),
    // so every step is branch-free: elements with j <= p are rewritten unchanged
    int ei[Q], ej[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int e = lane + WAVE * q;
        ei[q] = e < NE ? e / (n + 1) : n;
        ej[q] = e < NE ? e - (e / (n + 1)) * (n + 1) : n;
    }
#pragma unroll 1
    for (int p = 0; p < n; ++p) {
        // every read of the step is issued with the pivot's (one LDS round trip per step)
        const R d = M[p * LD + p];
        R mip[Q], mpj[Q], mij[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            mip[q] = M[ei[q] * LD + p];
            mpj[q] = M[p * LD + ej[q]];
            mij[q] = M[ei[q] * LD + ej[q]];
        }
        if (!(d > R(0))) return false;   // wave-uniform: every lane read the same pivot
        const R inv = rcp_nr(d);
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const R f = mpj[q] * inv;
            const R upd = ei[q] == p ? f : fma(-mip[q], f, mij[q]);
            M[ei[q] * LD + ej[q]] = ej[q] > p ? upd : mij[q];
        }
        wave_sync();
    }
    return true;
}

// The same Gauss-Jordan elimination with the rows in registers: lane i (< n) holds row i of [K + dw I | rhs] in
// a[0..n]; step p reads the pivot row's entries j > p by readlane (uniform), scales them by 1 / pivot and updates
// every other row — gj_lds's arithmetic element for element, without an LDS round trip per step (the steps are a
// readlane -> rcp -> fma chain).  On success lane i holds x_i in a[n].
template <int n, class R>
__device__ __forceinline__ bool gj_regs(R (&a)[n + 1], int lane)
{
    // r4: the pivot row is not normalised during the elimination (row i -= (a_ip / a_pp) row p for i != p; row p
    // stays), so no per-entry select between the pivot row and the others; the diagonal left at the end divides the
    // right-hand side once per lane.  The pivots a_pp are the same D of K = L D L^T (the positive-definiteness test).
#pragma unroll
    for (int p = 0; p < n; ++p) {
        const R d = bcast(a[p], p);
        if (!(d > R(0))) return false;   // wave-uniform
        const R m = lane == p ? R(0) : a[p] * rcp_nr(d);
#pragma unroll
        for (int j = p + 1; j <= n; ++j) a[j] = fma(-m, bcast(a[j], p), a[j]);
    }
    // lane i: x_i = a_i[n] / a_i[i]
    R dg = a[0];
#pragma unroll
    for (int i = 1; i < n; ++i) dg = lane == i ? a[i] : dg;
    a[n] = a[n] * rcp_nr(dg);
    return true;
}

// working copy for gj_lds: M[i][j] = K[i][j] + dw [i == j] (j <= n; column n = rhs), same element
// ownership as gj_lds (the padding element M[n][n] = 0)
template <int n, int LDK, int LD, class R>
__device__ __forceinline__ void gj_fill(const R* K, R* M, int lane, R dw)
{
    constexpr int NE = n * (n + 1), Q = (NE + WAVE - 1) / WAVE;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int e = lane + WAVE * q;
        const int i = e < NE ? e / (n + 1) : n, j = e < NE ? e - (e / (n + 1)) * (n + 1) : n;
        const R v = e < NE ? K[i * LDK + j] : R(0);
        M[i * LD + j] = v + (i == j && e < NE ? dw : R(0));
    }
}
template <int n, int LD, class R>
__device__ __forceinline__ void gj_zero(R* M, int lane)
{
    constexpr int NE = n * (n + 1), Q = (NE + WAVE - 1) / WAVE;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int e = lane + WAVE * q;
        const int i = e < NE ? e / (n + 1) : n, j = e < NE ? e - (e / (n + 1)) * (n + 1) : n;
        M[i * LD + j] = R(0);
    }
}

// ------------------------------------------------------------------------------------------------
// solve-kernel workspace.  Rows r < mr4 are the padded constraint rows; rows mr4 .. mr4+N-1 are the
// objective terms f_k (k = 1..N) treated as pseudo-rows ("OBJ rows"): same generator-form gradient, so
// grad f and J^T y come out of ONE J-layout sweep, and grad f . dV out of the row-layout dS pass.
// mo4 = mr4 + 4 ceil(N/4) rows in total.
// ------------------------------------------------------------------------------------------------
template <int N, class R>
struct WSS {
    typedef R real;
    R* V;      // NG   current generator values (canonical copy; rows keep register copies)
    R* Vt;     // NG   prologue scratch
    R* dV;     // NG   step
    R* CT;     // N+1  cos / sin of theta_k at V (written by the VBX rows, read by the Hessian lanes)
    R* ST;     // N+1
    R* S;      // (N+1) x 64 Hessian blocks
    R* hobj;   // (N+1) x 6 objective Hessian parts (written by the OBJ rows)
    R* rcoef;  // mo4 x 4
    R* cst;    // 16 per-instance constants read at use (keeps long-lived uniforms out of registers)
    R* ry;     // mo4   y (constraint rows), -1 (OBJ rows)
    R* rsig;   // mo4   Sigma
    R* rw;     // mo4   rhs weights (OBJ rows: -1)
    R* obs;    // prologue layout: circles 3*nc_max, ellipses 5*ne_max, then qa, qb, qc, ek (4*ne_max)
    R* obs6;   // (nc_max + ne_max) x 6 unified quadratic form [ox, oy, qa, qb, qc, ek] per row slot
    R* K;      // NCP x KLD
    R* rclo;   // mr4 original bounds (status / infeasibility checks only)
    R* rcuo;   // mr4
    int* nsel;      // [0] = nc_sel, [1] = ne_sel
    uint32_t* rgen; // mo4 packed generator indices (4 x 8 bit)
};

template <int N, class R>
__host__ __device__ constexpr int wss_elems(int nc_max, int ne_max, int mr4, int mo4)
{
    int d = 16 + 3 * Dim<N>::NG + 2 * (N + 1) + 64 * (N + 1) + 6 * (N + 1) + 4 * mo4 + 3 * mo4 + 3 * nc_max +
            9 * ne_max + 6 * (nc_max + ne_max) + 6 + Dim<N>::NCP * Dim<N>::KLD + 2 * mr4 +
            (int)(8 / sizeof(R)) + (int)((4 * mo4 + sizeof(R) - 1) / sizeof(R));
    return (d + 3) & ~3;   // 4-element multiple: rcoef rows (4 x R) are read as b128 (double: 2 x b128)
}

template <int N, class R>
__device__ WSS<N, R> carve_s(R* base, int nc_max, int ne_max, int mr4, int mo4)
{
    using D = Dim<N>;
    WSS<N, R> w;
    R* p = base;
    w.rcoef = p; p += 4 * mo4;   // first: 32-byte aligned
    w.cst = p; p += 16;
    w.V = p; p += D::NG;
    w.Vt = p; p += D::NG;
    w.dV = p; p += D::NG;
    w.CT = p; p += N + 1;
    w.ST = p; p += N + 1;
    w.S = p; p += 64 * (N + 1);
    w.hobj = p; p += 6 * (N + 1);
    w.ry = p; p += mo4;
    w.rsig = p; p += mo4;
    w.rw = p; p += mo4;
    w.obs = p; p += 3 * nc_max + 9 * ne_max;
    w.obs6 = p; p += 6 * (nc_max + ne_max) + 6;
    w.K = p; p += D::NCP * D::KLD;
    w.rclo = p; p += mr4;
    w.rcuo = p; p += mr4;
    w.nsel = reinterpret_cast<int*>(p); p += 8 / sizeof(R);
    w.rgen = reinterpret_cast<uint32_t*>(p);
    return w;
}

// generator rows a row reads: VEL rows [vx, vy, theta of x_{k+1}, turn p_k], obstacle rows
// [px, py of x_{k+1}, px, py of x_k], LEG [px, py of x_k, foot x, y of p_k], DTH [-, -, -, turn p_k],
// OBJ [px, py, theta of x_k, -]
__device__ __forceinline__ uint32_t row_gens(int type, int k)
{
    int g0 = 0, g1 = 0, g2 = 0, g3 = 0;
    switch (type) {
    case R_VBX:
    case R_VBY:
    case R_FEN:
    case R_FENM:
        g0 = gx(k + 1, 2); g1 = gx(k + 1, 3); g2 = gx(k + 1, 4); g3 = gp(k, 2);
        break;
    case R_CIR:
    case R_ELP:
        g0 = gx(k + 1, 0); g1 = gx(k + 1, 1); g2 = gx(k, 0); g3 = gx(k, 1);
        break;
    case R_LEG:
        g0 = gx(k, 0); g1 = gx(k, 1); g2 = gp(k, 0); g3 = gp(k, 1);
        break;
    case R_DTH:
        g3 = gp(k, 2);
        break;
    case R_OBJ:
        g0 = gx(k, 0); g1 = gx(k, 1); g2 = gx(k, 4);
        break;
    default:
        break;
    }
    return (uint32_t)g0 | ((uint32_t)g1 << 8) | ((uint32_t)g2 << 16) | ((uint32_t)g3 << 24);
}

__device__ __forceinline__ int gen_i(uint32_t pk, int i) { return (int)((pk >> (8 * i)) & 255u); }

// the transcendental part of a row: VEL rows sincos(theta_{k+1}) -> (a0, a1) = (sin, cos);
// OBJ rows phi = theta_k - atan2(goal - p) -> a0.  (Computed for every lane; lanes keep what they need.)
template <class R>
__device__ __forceinline__ void row_trans(int type, const R (&v)[4], R gxg, R gyg, R& a0, R& a1)
{
    R s_, c_;
    lsincos(v[2], &s_, &c_);
    const R at = latan2(gyg - v[1], gxg - v[0]);
    a0 = type == R_OBJ ? v[2] - at : s_;
    a1 = c_;
}

template <class R>
struct RowK {   // uniform constants of the row functions
    R gm1, s, q, p, r, gxg, gyg;
};
// cst slots
enum { K_GM1 = 0, K_S, K_Q, K_P, K_R, K_GXG, K_GYG, K_THMAX, K_THMIN, K_MACT, K_NBL, K_TOL, K_ACCTOL, K_NTR, K_XR };
template <class R>
__device__ __forceinline__ RowK<R> load_rowk(const R* cst)
{
    RowK<R> C;
    C.gm1 = cst[K_GM1]; C.s = cst[K_S]; C.q = cst[K_Q]; C.p = cst[K_P]; C.r = cst[K_R];
    C.gxg = cst[K_GXG]; C.gyg = cst[K_GYG];
    return C;
}

// value of row `type` at generator values v (branch-free: every family is computed, one is selected)
template <class R>
__device__ __forceinline__ R row_value(int type, int k, const R (&v)[4], R a0, R a1,
                                            const R (&o)[6], const RowK<R>& C)
{
    // velocity family (f_en halves: vbx +- s dth)
    const bool vby = type == R_VBY;
    const R ca = vby ? -a0 : a1, cb = vby ? a1 : a0;
    const R sd = type == R_FEN ? C.s : (type == R_FENM ? -C.s : R(0));
    const R cvel = ca * v[0] + cb * v[1] + sd * v[3];
    // D-CBF (circle == ellipse with qa = qc = 1, qb = 0, ek = r^2)
    const R x1 = v[0] - o[0], y1 = v[1] - o[1], x0 = v[2] - o[0], y0 = v[3] - o[1];
    const R h1 = o[2] * x1 * x1 + o[3] * x1 * y1 + o[4] * y1 * y1 - o[5];
    const R h0 = o[2] * x0 * x0 + o[3] * x0 * y0 + o[4] * y0 * y0 - o[5];
    const R cobs = h1 + C.gm1 * h0;
    // leg length
    const R ex = v[0] - v[2], ey = v[1] - v[3];
    const R cleg = ex * ex + ey * ey;
    // objective term f_k
    const R w = C.q + (k == 1 ? C.p : R(0));
    const R dxg = C.gxg - v[0], dyg = C.gyg - v[1];
    const R cobj = w * (dxg * dxg + dyg * dyg) + C.r * a0 * a0;
    R c = R(0);
    c = (type == R_VBX || vby || type == R_FEN || type == R_FENM) ? cvel : c;
    c = (type == R_CIR || type == R_ELP) ? cobs : c;
    c = type == R_LEG ? cleg : c;
    c = type == R_DTH ? v[3] : c;
    c = type == R_OBJ ? cobj : c;
    return c;
}

// generator-form gradient coefficients of row `type` (OBJ rows: grad f_k; hx = its 6 Hessian parts
// [h00 h01 h11 h04 h14 h44] on (px, py, theta) of x_k)
template <class R>
__device__ __forceinline__ void row_coef(int type, int k, const R (&v)[4], R a0, R a1,
                                         const R (&o)[6], const RowK<R>& C, R (&cf)[4], R (&hx)[6])
{
    const bool vby = type == R_VBY, vel = type == R_VBX || vby || type == R_FEN || type == R_FENM;
    const bool obs = type == R_CIR || type == R_ELP;
    // velocity family: d/dtheta of (ca, cb)
    const R ca = vby ? -a0 : a1, cb = vby ? a1 : a0;
    const R da = vby ? -a1 : -a0, db = vby ? -a0 : a1;
    // D-CBF
    const R x1 = v[0] - o[0], y1 = v[1] - o[1], x0 = v[2] - o[0], y0 = v[3] - o[1];
    // leg
    const R ex = v[0] - v[2], ey = v[1] - v[3];
    // objective
    const R w = C.q + (k == 1 ? C.p : R(0));
    const R dxg = C.gxg - v[0], dyg = C.gyg - v[1];
    // (at p = goal exactly the target heading atan2(0, 0) = 0 is taken as locally constant: DESIGN.md §2 item 7)
    const R rho2 = dxg * dxg + dyg * dyg, ir2 = rho2 > R(0) ? rcp_nr(rho2) : R(0);
    const R gp0 = -dyg * ir2, gp1 = dxg * ir2, phi = a0;
    R c0 = R(0), c1 = R(0), c2 = R(0), c3 = R(0);
    if (vel) {
        c0 = ca; c1 = cb; c2 = da * v[0] + db * v[1]; c3 = type == R_FEN ? C.s : (type == R_FENM ? -C.s : R(0));
    }
    if (obs) {
        c0 = 2 * o[2] * x1 + o[3] * y1; c1 = 2 * o[4] * y1 + o[3] * x1;
        c2 = C.gm1 * (2 * o[2] * x0 + o[3] * y0); c3 = C.gm1 * (2 * o[4] * y0 + o[3] * x0);
    }
    if (type == R_LEG) {
        c0 = 2 * ex; c1 = 2 * ey; c2 = -2 * ex; c3 = -2 * ey;
    }
    if (type == R_DTH) c3 = R(1);
    if (type == R_OBJ) {
        c0 = -2 * w * dxg + 2 * C.r * phi * gp0;
        c1 = -2 * w * dyg + 2 * C.r * phi * gp1;
        c2 = 2 * C.r * phi;
        const R ir4 = ir2 * ir2;
        const R s00 = 2 * dxg * dyg * ir4, s01 = (dyg * dyg - dxg * dxg) * ir4, s11 = -2 * dxg * dyg * ir4;
        hx[0] = 2 * w + 2 * C.r * (gp0 * gp0 - phi * s00);
        hx[1] = 2 * C.r * (gp0 * gp1 - phi * s01);
        hx[2] = 2 * w + 2 * C.r * (gp1 * gp1 - phi * s11);
        hx[3] = 2 * C.r * gp0;
        hx[4] = 2 * C.r * gp1;
        hx[5] = 2 * C.r;
    }
    cf[0] = c0; cf[1] = c1; cf[2] = c2; cf[3] = c3;
}

// ------------------------------------------------------------------------------------------------
// Hessian blocks of L = f - y^T c: lane kb (0..N) writes S block kb (8x8, symmetric).  Objective parts
// come from the OBJ rows (hobj), everything else from y and the obstacle forms.
// ------------------------------------------------------------------------------------------------
template <int N, class R>
__device__ void hess_blocks(const WSS<N, R>& w, int lane, int rps, int nobs, int modi)
{
    if (lane > N) return;
    const R gm1 = w.cst[K_GM1];
    const int kb = lane;
    R h00 = 0, h01 = 0, h11 = 0, h04 = 0, h14 = 0, h44 = 0, h24 = 0, h34 = 0;
    R h05 = 0, h55 = 0;
    if (kb >= 1) {
        const R* ho = w.hobj + 6 * kb;
        h00 = ho[0]; h01 = ho[1]; h11 = ho[2]; h04 = ho[3]; h14 = ho[4]; h44 = ho[5];
        // rows of step kb-1 act on x_kb as the post-step state
        const int base = (kb - 1) * rps;
        const R ct = w.CT[kb], st = w.ST[kb];
        const R vx = w.V[gx(kb, 2)], vy = w.V[gx(kb, 3)];
        const R vbx = ct * vx + st * vy, vby = -st * vx + ct * vy;
        const R wbx = w.ry[base + 0] + (modi ? w.ry[base + rps - 2] + w.ry[base + rps - 1] : R(0));
        const R wby = w.ry[base + 1];
        h24 = wbx * st + wby * ct;
        h34 = -wbx * ct + wby * st;
        h44 += wbx * vbx + wby * vby;
        // inactive slots have y = 0 and a zero form
#pragma unroll 4
        for (int j = 0; j < nobs; ++j) {
            const R y = w.ry[base + 2 + j];
            const R* o = w.obs6 + 6 * j;
            h00 -= 2 * y * o[2];
            h01 -= y * o[3];
            h11 -= 2 * y * o[4];
        }
    }
    if (kb < N) {
        const int base = kb * rps;
        if (kb >= 1) {
#pragma unroll 4
            for (int j = 0; j < nobs; ++j) {
                const R y = w.ry[base + 2 + j] * gm1;
                const R* o = w.obs6 + 6 * j;
                h00 -= 2 * y * o[2];
                h01 -= y * o[3];
                h11 -= 2 * y * o[4];
            }
        }
        const R yl = w.ry[base + 2 + nobs];
        h00 -= 2 * yl;
        h11 -= 2 * yl;
        h05 = 2 * yl;
        h55 = -2 * yl;
    }
    R* S = w.S + 64 * kb;
    S[0 * 8 + 0] = h00; S[0 * 8 + 1] = h01; S[1 * 8 + 0] = h01; S[1 * 8 + 1] = h11;
    S[0 * 8 + 4] = h04; S[4 * 8 + 0] = h04; S[1 * 8 + 4] = h14; S[4 * 8 + 1] = h14;
    S[2 * 8 + 4] = h24; S[4 * 8 + 2] = h24; S[3 * 8 + 4] = h34; S[4 * 8 + 3] = h34; S[4 * 8 + 4] = h44;
    S[0 * 8 + 5] = h05; S[5 * 8 + 0] = h05; S[1 * 8 + 6] = h05; S[6 * 8 + 1] = h05;
    S[5 * 8 + 5] = h55; S[6 * 8 + 6] = h55;
}

// sum over each 16-lane DPP row (every lane of the row receives its row's sum)
template <class T>
__device__ __forceinline__ T rsum16(T v)
{
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    v += dpp<0x141>(v);
    v += dpp<0x140>(v);
    return v;
}

// hess_blocks with the obstacle terms spread over lanes (16 (N + 1) <= 64 lanes): lane 16 kb + j takes
// obstacle slots j and j + 16's terms on block kb — the post-step state of step kb - 1 and the pre-step state of step kb, whose
// multipliers combine as y_post + gamma_1 y_pre on the same form — and each block's sum is one 16-lane DPP reduction.
// The serial form above walks the slots with one dependent LDS round trip per unrolled group: on a lone wave that
// phase had cost 3.2 k of the 22 k cycles of an iteration (tools/stamps.py, profiles/r5).  The same terms, summed in
// another order (rounding-level differences only).
template <int N, class R>
__device__ void hess_blocks_lanes(const WSS<N, R>& w, int lane, int rps, int nobs, int modi)
{
    static_assert(16 * (N + 1) <= WAVE, "one 16-lane row per block");
    static_assert(ALIPMPC_MAX_OBS <= 32, "lane j takes obstacle slots j and j + 16 only (ADVICE r5)");
    const int kb = lane >> 4, j = lane & 15;
    const R gm1 = w.cst[K_GM1];
    R t00 = R(0), t01 = R(0), t11 = R(0);
    // slots j and j + 16 (ALIPMPC_MAX_OBS = 24); inactive slots have y = 0 and a zero form
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int js = j + 16 * h;
        if (kb >= 1 && kb <= N && js < nobs) {
            const R* o = w.obs6 + 6 * js;
            R y = w.ry[(kb - 1) * rps + 2 + js];
            if (kb < N) y = fma(w.ry[kb * rps + 2 + js], gm1, y);
            t00 = fma(R(-2) * y, o[2], t00);
            t01 = fma(-y, o[3], t01);
            t11 = fma(R(-2) * y, o[4], t11);
        }
    }
    const R a00 = rsum16(t00), a01 = rsum16(t01), a11 = rsum16(t11);
    if (j != 0 || kb > N) return;
    R h00 = 0, h01 = 0, h11 = 0, h04 = 0, h14 = 0, h44 = 0, h24 = 0, h34 = 0;
    R h05 = 0, h55 = 0;
    if (kb >= 1) {
        const R* ho = w.hobj + 6 * kb;
        h00 = ho[0] + a00; h01 = ho[1] + a01; h11 = ho[2] + a11; h04 = ho[3]; h14 = ho[4]; h44 = ho[5];
        const int base = (kb - 1) * rps;
        const R ct = w.CT[kb], st = w.ST[kb];
        const R vx = w.V[gx(kb, 2)], vy = w.V[gx(kb, 3)];
        const R vbx = ct * vx + st * vy, vby = -st * vx + ct * vy;
        const R wbx = w.ry[base + 0] + (modi ? w.ry[base + rps - 2] + w.ry[base + rps - 1] : R(0));
        const R wby = w.ry[base + 1];
        h24 = wbx * st + wby * ct;
        h34 = -wbx * ct + wby * st;
        h44 += wbx * vbx + wby * vby;
    }
    if (kb < N) {
        const R yl = w.ry[kb * rps + 2 + nobs];
        h00 -= 2 * yl;
        h11 -= 2 * yl;
        h05 = 2 * yl;
        h55 = -2 * yl;
    }
    R* S = w.S + 64 * kb;
    S[0 * 8 + 0] = h00; S[0 * 8 + 1] = h01; S[1 * 8 + 0] = h01; S[1 * 8 + 1] = h11;
    S[0 * 8 + 4] = h04; S[4 * 8 + 0] = h04; S[1 * 8 + 4] = h14; S[4 * 8 + 1] = h14;
    S[2 * 8 + 4] = h24; S[4 * 8 + 2] = h24; S[3 * 8 + 4] = h34; S[4 * 8 + 3] = h34; S[4 * 8 + 4] = h44;
    S[0 * 8 + 5] = h05; S[5 * 8 + 0] = h05; S[1 * 8 + 6] = h05; S[6 * 8 + 1] = h05;
    S[5 * 8 + 5] = h55; S[6 * 8 + 6] = h55;
}

// ------------------------------------------------------------------------------------------------
// the solve kernel: one instance per wave.
//   Row layout (lane r = row r [+ 64]): values, multipliers, slacks, bound terms, and a REGISTER copy of
//   the 4 generator values each row reads (rv) and of their step (rdv), so line-search trial points
//   V + a dV are evaluated without touching LDS.  The canonical V lives in LDS (lane t owns V[t]).
//   J layout (lane = (g4, col), rows 4s + g4, KSM steps, fully unrolled): J^T y, grad f, J^T w and the
//   MFMA KKT products.
// ------------------------------------------------------------------------------------------------
// sum of the N objective pseudo-rows (rows mr4 .. mr4 + N - 1) of a row-layout value, in step order (the
// oracle's order): N readlanes instead of a 64-lane reduction
template <int N, int RPL, class R>
__device__ __forceinline__ R obj_sum(const R (&v)[RPL], int mr4)
{
    R s = R(0);
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const int r = mr4 + k, q = r / WAVE, l = r - q * WAVE;
        R x = v[0];
#pragma unroll
        for (int qq = 1; qq < RPL; ++qq) x = q == qq ? v[qq] : x;
        s += bcast(x, l);
    }
    return s;
}

// team hand-over of the winning trial's values through LDS (instead of every other member re-evaluating it): when
// they fit the KKT area of a workspace (3 row values per row slot + 3 scalars), which every iteration rewrites in
// full before reading it (the Hessian-block area keeps a zero pattern across iterations, so not that one)
template <int N, int RPL>
constexpr bool TEAM_HANDOVER = 3 * WAVE * RPL + 3 <= Dim<N>::NCP * Dim<N>::KLD;

#include "resto_wave.inc"

// TM: the team-capable build (split launches with team records, solve_kernel<..., TM = true>): phase 1 also cuts an
// instance by its line-search trial count, phase 2 runs team records on 4 waves; tm < 0 = member -1 - tm of a team.
// Without TM all of it compiles out: the interior-point loop of the plain build sits at its register budget, and the
// team logic in the same body had cost 36 -> 172 B/lane of spills (the register allocator, not the arithmetic).
// RS: the restoration-capable build (cfg.restoration = IPOPT): a failed line search runs IPOPT's restoration phase
// (resto_wave.inc, inlined) at the top of the next iteration.  The lean build (RS = false: phase 1 of a split launch)
// instead cuts the instance to a split record flagged "restoration pending", and phase 2's RS build runs the phase
// first — so the restoration's registers never touch the lean loop that most instances finish in.
template <int N, int KSM, class R, bool Q, bool TM = false, bool RS = false>
__device__ __forceinline__ void solve_one(const KP& P0, R* G, R* wsb, int wv, long long b, long long rec = -1,
                                          int tm = 0)
{
    if constexpr (!TM) tm = 0;
    // Q (persistent instance loop): opaque per-instance copies of the lane-/wave-derived inputs, so that
    // nothing computed from them is loop-invariant and no address or row table is hoisted out of the
    // instance loop (and spilled).  (Laundering the LDS base offsets as well cut the scratch further but
    // measured slower: profiles/r1f/ab_occupancy.log.)
    if constexpr (Q) asm volatile("" : "+s"(wv), "+s"(b));
    const KP& P = P0;
    using D = Dim<N>;
    constexpr int n = D::n;
    constexpr int NT = D::NT;
    constexpr int NCP = D::NCP;
    constexpr int NG = D::NG;
    constexpr int KLD = D::KLD;
    constexpr int RPL = (4 * KSM + WAVE - 1) / WAVE;
    constexpr bool JC = KSM * NT <= 16;   // keep the J tile in registers between the two J-layout passes
    constexpr bool GJ = n <= ALIP_GJ_MAX_N;   // KKT solve: Gauss-Jordan (small n) or register Cholesky
    constexpr int GJLD = n + 1;           // row stride of the Gauss-Jordan working copy (in the S buffer)
    constexpr bool GJ_REGS = ALIP_GJ_REGS != 0;   // Gauss-Jordan on register rows (gj_regs) instead of LDS
    static_assert((n + 1) * (n + 1) <= 64 * (N + 1), "GJ working copy fits the S-block buffer");
    static_assert(NG <= WAVE, "one generator row per lane");
    int lane = lane_id();
    if constexpr (Q) RELAUNDER(lane);
#ifndef ALIP_NO_SETPRIO
    __builtin_amdgcn_s_setprio(0);   // a persistent wave starts each instance at base priority
#endif
    // uniform problem sizes in SGPRs (P lives in LDS: a plain read would be a per-lane VGPR value)
    const int mr4 = rfl(P.mr4), mo4 = rfl(P.mo4), m_max = rfl(P.m_max), rps = rfl(P.rps);
    const int nc_max = rfl(P.nc_max), ne_max = rfl(P.ne_max), nobs = nc_max + ne_max;
    const int modi = rfl(P.modi), max_iter = rfl(P.max_iter);
    WSTAMP_DECL
    WSS<N, R> w = carve_s<N, R>(wsb + (size_t)wv * wss_elems<N, R>(nc_max, ne_max, mr4, mo4), nc_max, ne_max, mr4, mo4);
    for (int i = lane; i < 64 * (N + 1); i += WAVE) w.S[i] = R(0.0);
    // tm < 0: member -1 - tm of a team (team-capable build).  The line-search trial count (phase 1's trial cut,
    // w.cst[K_NTR]) and a team's exchange-round parity (w.cst[K_XR]) live in LDS, not in loop-carried registers

    double gxg, gyg, uj;
    int legv;
    prologue<N>(P, w, G, P.E, b, gxg, gyg, legv, uj);   // (E from global memory: read once per instance)
    const int nc_sel = w.nsel[0], ne_sel = w.nsel[1];
    // unified quadratic forms per obstacle row slot (zero form for unused slots)
    {
        for (int j = lane; j <= nobs; j += WAVE) {
            R o[6] = {0, 0, 0, 0, 0, 0};
            if (j < nc_max) {
                if (j < nc_sel) {
                    const R* c = w.obs + 3 * j;
                    o[0] = c[0]; o[1] = c[1]; o[2] = R(1.0); o[4] = R(1.0); o[5] = c[2] * c[2];
                }
            } else if (j < nobs) {
                const int e = j - nc_max;
                if (e < ne_sel) {
                    const R* el = w.obs + 3 * nc_max + 5 * e;
                    const R* qq = w.obs + 3 * nc_max + 5 * ne_max;
                    o[0] = el[0]; o[1] = el[1];
                    o[2] = qq[e]; o[3] = qq[ne_max + e]; o[4] = qq[2 * ne_max + e]; o[5] = qq[3 * ne_max + e];
                }
            }
#pragma unroll
            for (int i = 0; i < 6; ++i) w.obs6[6 * j + i] = o[i];
        }
    }
    int g4 = lane >> 4, col = lane & 15;
    // per-row bound flags are recomputed at use (hoisted lane masks would pin ~2 SGPRs each)
#define HL(q) (cl[q] != -INFINITY)
#define HU(q) (cu[q] != INFINITY)
#define RELANE()                        \
    do {                                \
        RELAUNDER(lane);                \
        g4 = lane >> 4;                 \
        col = lane & 15;                \
        for (int q_ = 0; q_ < RPL; ++q_) { \
            RELAUNDER(rtype[q_]);       \
            RELAUNDER(rk[q_]);          \
            RELAUNDER(roi[q_]);         \
            RELAUNDER(rg[q_]);          \
            RELAUNDER(cl[q_]);          \
            RELAUNDER(cu[q_]);          \
        }                               \
    } while (0)
    if (lane == 0) {
        w.cst[K_NTR] = R(0.0);
        w.cst[K_XR] = R(0.0);
        w.cst[K_GM1] = P.gm1; w.cst[K_S] = P.s; w.cst[K_Q] = P.q; w.cst[K_P] = P.p; w.cst[K_R] = P.r;
        w.cst[K_GXG] = gxg; w.cst[K_GYG] = gyg; w.cst[K_TOL] = P.tol; w.cst[K_ACCTOL] = P.acc_tol;
    }
    wave_sync();
#define CK load_rowk(w.cst)

    // ---- per-row state (registers)
    int rtype[RPL], rk[RPL], roi[RPL];
    uint32_t rg[RPL];
    R cl[RPL], cu[RPL], rv[RPL][4], rdv[RPL][4], ra0[RPL], ra1[RPL];
    R cr[RPL], sr[RPL], zl[RPL], zu[RPL], idl[RPL], idu[RPL];
    R mu = uni(R(P.mu_init));
    R vme = lane < NG ? w.V[lane] : R(0.0), dvme = R(0.0);   // lane t's generator value / step
    R th0 = R(0.0), nbl = R(0.0), mal = R(0.0), fo = R(0.0), lg0 = R(0.0);
    wave_sync();
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
        const int r = lane + WAVE * q;
        RowInfo ri;
        ri.type = R_NONE; ri.k = 0; ri.slot = 0;
        if (r < m_max) {
            ri = decode_row(P, r, nc_sel, ne_sel);
        } else if (r >= mr4 && r < mr4 + N) {
            ri.type = R_OBJ;
            ri.k = r - mr4 + 1;
        }
        rtype[q] = ri.type;
        rk[q] = ri.k;
        roi[q] = ri.type == R_CIR ? ri.slot : (ri.type == R_ELP ? nc_max + ri.slot : 0);
        rg[q] = row_gens(ri.type, ri.k);
        if (r < mo4) w.rgen[r] = rg[q];
        R clo, cuo;
        row_bounds(P, ri, legv, clo, cuo, modi != 0);
        if (r < mr4) {
            w.rclo[r] = clo;
            w.rcuo[r] = cuo;
        }
        nbl += (R)isfinite(clo) + (R)isfinite(cuo);
        mal += ri.type < R_NONE ? R(1.0) : R(0.0);
        cl[q] = isfinite(clo) ? clo - R(1e-8) * fmax(R(1.0), fabs(clo)) : -INFINITY;
        cu[q] = isfinite(cuo) ? cuo + R(1e-8) * fmax(R(1.0), fabs(cuo)) : INFINITY;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            rv[q][i] = w.V[gen_i(rg[q], i)];
            rdv[q][i] = R(0.0);
        }
        R o[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) o[i] = w.obs6[6 * roi[q] + i];
        row_trans(rtype[q], rv[q], w.cst[K_GXG], w.cst[K_GYG], ra0[q], ra1[q]);
        cr[q] = row_value(rtype[q], rk[q], rv[q], ra0[q], ra1[q], o, CK);
        R v = cr[q];
        const R pl = HL(q) ? fmin(R(1e-2) * fmax(R(1.0), fabs(cl[q])), R(1e-2) * (cu[q] - cl[q])) : R(0.0);
        const R pu = HU(q) ? fmin(R(1e-2) * fmax(R(1.0), fabs(cu[q])), R(1e-2) * (cu[q] - cl[q])) : R(0.0);
        if (HL(q) && HU(q))
            v = fmin(fmax(v, cl[q] + pl), cu[q] - pu);
        else if (HL(q))
            v = fmax(v, cl[q] + pl);
        else if (HU(q))
            v = fmin(v, cu[q] - pu);
        sr[q] = rtype[q] < R_NONE ? v : R(0.0);
        zl[q] = HL(q) ? R(1.0) : R(0.0);
        zu[q] = HU(q) ? R(1.0) : R(0.0);
        const R dl = sr[q] - cl[q], du = cu[q] - sr[q];
        idl[q] = HL(q) ? R(1.0) / dl : R(0.0);
        idu[q] = HU(q) ? R(1.0) / du : R(0.0);
        lg0 += llog(HL(q) ? (HU(q) ? dl * du : dl) : (HU(q) ? du : R(1.0)));   // (one log per lane: log 1 = 0)
        if (rtype[q] < R_NONE) th0 += fabs(cr[q] - sr[q]);
    }
    wsum2(th0, nbl);
    lg0 = wsum(lg0);
    // IPOPT's default NLP scaling at the starting point (nlp_scaling_method = gradient-based; the reference sets no
    // scaling option, MPC_LIP_modi.py:274-296): the OBJ rows' gradient on (px, py, theta) of x_k, taken to the
    // reference's u through Gu (d x_k / d u), and the objective scaled by 100 / max |grad f| where that exceeds 100 —
    // the objective is linear in its weights, so the weights are scaled (constraint rows' gradients stay below 4 in u on
    // every benchmark scene and exceed 100 only with select_obs = 0 and large distant ellipses: no row scaling, a
    // stated deviation)
    {
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            if (rtype[q] == R_OBJ) {
                R o[6] = {R(0), R(0), R(0), R(0), R(0), R(0)}, cf[4], hx[6];
                row_coef(R_OBJ, rk[q], rv[q], ra0[q], ra1[q], o, CK, cf, hx);
                const int k = rk[q] - 1;
                w.Vt[3 * k] = cf[0];
                w.Vt[3 * k + 1] = cf[1];
                w.Vt[3 * k + 2] = cf[2];
            }
        }
        wave_sync();
        R gu = R(0);
        if (lane < D::nu) {
#pragma unroll
            for (int k = 1; k <= N; ++k) {
                const double* gr = P.Gu + (size_t)(8 * k) * D::NCPU + lane;
                gu += w.Vt[3 * (k - 1)] * (R)gr[0] + w.Vt[3 * (k - 1) + 1] * (R)gr[D::NCPU] +
                      w.Vt[3 * (k - 1) + 2] * (R)gr[4 * D::NCPU];
            }
        }
        const R gm = wmax(fabs(gu));
#ifdef ALIP_NO_OBJ_SCALING   // dev A/B timing only (changes the algorithm where the gradient exceeds 100)
        const R dfo = R(1);
#else
        const R dfo = uni(gm > R(100) ? fmax(R(1e-8), R(100) / gm) : R(1));
#endif
        wave_sync();
        if (dfo != R(1)) {
            if (lane == 0) {
                w.cst[K_Q] *= dfo;
                w.cst[K_P] *= dfo;
                w.cst[K_R] *= dfo;
            }
#pragma unroll
            for (int q = 0; q < RPL; ++q)
                if (rtype[q] == R_OBJ) cr[q] *= dfo;
            wave_sync();
        }
    }
    fo = obj_sum<N, RPL>(cr, mr4);
    mal = wsum(mal);
    R f_cur = fo, lsum_cur = lg0;
    if (lane == 0) {
        w.cst[K_THMAX] = R(1e4) * fmax(R(1.0), th0);
        w.cst[K_THMIN] = R(1e-4) * fmax(R(1.0), th0);
        w.cst[K_MACT] = mal;
        w.cst[K_NBL] = nbl;
    }
    wave_sync();
    R fth0 = INFINITY, fph0 = INFINITY, fth1 = INFINITY, fph1 = INFINITY;   // filter entries lane, lane+64
    int nf = 0;
    R dw_last = R(0.0);
    int status = -1, it = 0, n_rest = 0;
    // Error_In_Step_Computation: iteration (+ FAIL_GOAL: Invalid_Number_Detected), and the loop's end
    int fail_it = -1, it_end = max_iter;
    R e0 = INFINITY;
    R theta_c = R(0.0);
    bool theta_ok = false;
    // restoration pending (cfg.restoration = IPOPT): the line search of the last iteration failed at the current point,
    // whose violation theta_R entered the filter
    bool rpend = false;
    R theta_R = R(0.0);
    const R gth = R(1e-5), gph = R(1e-8), sth = R(1.1), sph = R(2.3), eta = R(1e-8), gal = R(0.05);

    int it0 = 0;
    if (rec >= 0) {
        // split launch, phase 2: the loop state at the top of iteration `it`, from the record phase 1 wrote (all
        // of it: values the loop could recompute are stored too, so no recomputation can round differently).
        const double* rc = P.ckpt + rec * ckpt_doubles(mo4);
        const double* sc = rc + ck_scal(mo4);
        nf = rfl((int)sc[5]);
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int r = lane + WAVE * q;
            if (r < mo4) {   // (rows r >= mo4 keep the prologue's values: no row there)
                const double* rq = rc + r;
                sr[q] = ck_get<R>(rq[0]);
                zl[q] = ck_get<R>(rq[mo4]);
                zu[q] = ck_get<R>(rq[2 * mo4]);
                idl[q] = ck_get<R>(rq[3 * mo4]);
                idu[q] = ck_get<R>(rq[4 * mo4]);
                cr[q] = ck_get<R>(rq[5 * mo4]);
                ra0[q] = ck_get<R>(rq[6 * mo4]);
                ra1[q] = ck_get<R>(rq[7 * mo4]);
#pragma unroll
                for (int i = 0; i < 4; ++i) rv[q][i] = ck_get<R>(rq[(8 + i) * mo4]);
            }
        }
        const double* rf = rc + ck_filt(mo4) + lane;   // (entries >= nf are never read by the filter tests)
        if (lane < nf) {
            fth0 = ck_get<R>(rf[0]);
            fph0 = ck_get<R>(rf[2 * WAVE]);
        }
        if (lane + WAVE < nf) {
            fth1 = ck_get<R>(rf[WAVE]);
            fph1 = ck_get<R>(rf[3 * WAVE]);
        }
        vme = lane < NG ? ck_get<R>(rc[ck_vme(mo4) + lane]) : R(0.0);
        mu = uni(ck_get<R>(sc[0]));
        f_cur = uni(ck_get<R>(sc[1]));
        lsum_cur = uni(ck_get<R>(sc[2]));
        theta_c = uni(ck_get<R>(sc[3]));
        dw_last = uni(ck_get<R>(sc[4]));
        it0 = rfl((int)sc[6]);
        n_rest = rfl((int)sc[7]);
        fail_it = rfl((int)sc[8]);
        it_end = rfl((int)sc[9]);
        theta_ok = rfl((int)sc[10]) != 0;
        if constexpr (RS) {   // (a lean-build record: the restoration pending at its point)
            rpend = rfl((int)sc[11]) != 0;
            theta_R = uni(ck_get<R>(sc[12]));
        }
        if (lane < NG) w.V[lane] = vme;
        wave_sync();
#ifndef ALIP_NO_SETPRIO
        // (a team is the critical path of its launch by construction — the instance whose line searches ran long —
        // and in the closed loop it shares SIMDs with the other episode group's phase 1: top priority)
        if (it0 >= 20 || (TM && tm < 0))
            __builtin_amdgcn_s_setprio(3);
        else if (it0 >= 14)
            __builtin_amdgcn_s_setprio(2);
        else if (it0 >= 8)
            __builtin_amdgcn_s_setprio(1);
#endif
    }

    // phase-1 cuts (a team's own solve is never cut)
    const int ckpt_it = TM && tm < 0 ? 0 : rfl(P.ckpt_it);
    const int ckpt_tr = TM && tm >= 0 ? rfl(P.team > 0 ? P.ckpt_tr : 0) : 0;
    STAMP_DECL
    // the loop state as a split record (record k of the launch): phase 2 resumes it exactly (rp: a restoration is
    // pending at this point, theta_R its violation)
    auto put_record = [&](bool to_team, bool rp) {
        int k = 0;
        if (lane == 0)
            k = to_team ? (int)(P.B - 1 - (long long)atomicAdd(P.cont + CONT_TEAM, 1u))
                        : (int)atomicAdd(P.cont + CONT_SINGLE, 1u);
        k = rfl(k);
        double* rc = P.ckpt + (long long)k * ckpt_doubles(mo4);
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int r = lane + WAVE * q;
            if (r < mo4) {
                double* rq = rc + r;
                rq[0] = ck_put(sr[q]);
                rq[mo4] = ck_put(zl[q]);
                rq[2 * mo4] = ck_put(zu[q]);
                rq[3 * mo4] = ck_put(idl[q]);
                rq[4 * mo4] = ck_put(idu[q]);
                rq[5 * mo4] = ck_put(cr[q]);
                rq[6 * mo4] = ck_put(ra0[q]);
                rq[7 * mo4] = ck_put(ra1[q]);
#pragma unroll
                for (int i = 0; i < 4; ++i) rq[(8 + i) * mo4] = ck_put(rv[q][i]);
            }
        }
        double* rf = rc + ck_filt(mo4) + lane;
        if (lane < nf) {
            rf[0] = ck_put(fth0);
            rf[2 * WAVE] = ck_put(fph0);
        }
        if (lane + WAVE < nf) {
            rf[WAVE] = ck_put(fth1);
            rf[3 * WAVE] = ck_put(fph1);
        }
        if (lane < NG) rc[ck_vme(mo4) + lane] = ck_put(vme);
        const double sv[13] = {ck_put(mu), ck_put(f_cur), ck_put(lsum_cur), ck_put(theta_c), ck_put(dw_last),
                               (double)nf, (double)it, (double)n_rest, (double)fail_it, (double)it_end,
                               theta_ok ? 1.0 : 0.0, rp ? 1.0 : 0.0, ck_put(theta_R)};
        double v = 0.0;
#pragma unroll
        for (int i = 0; i < 13; ++i) v = lane == i ? sv[i] : v;
        if (lane < 13) rc[ck_scal(mo4) + lane] = v;
        if (lane == 0) P.cont[cont_hdr(P.B) + k] = (uint32_t)b;
    };
    R phi_R = R(0.0);
    it = it0;
    // regular iterations; with cfg.restoration = IPOPT a failed line search leaves this loop (ST_RESTO) and IPOPT's
    // restoration phase runs between two passes of it (RS build) or in phase 2 (the lean build cuts the instance)
    for (;;) {
    if constexpr (RS) {
        if (rpend) {
            // IPOPT's restoration phase from the failed point (the current iterate, slacks and multipliers; the
            // augmented filter; theta_R), resto_wave.inc; its iterate comes back through the workspace
            rpend = false;
            STAMP(8);
            RELANE();
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                const int r = lane + WAVE * q;
                if (r < mo4) {
                    w.ry[r] = sr[q];
                    w.rsig[r] = zl[q];
                    w.rw[r] = zu[q];
                }
            }
            if (lane < NG) w.V[lane] = vme;
            wave_sync();
            const int rr = rfl(resto_wave<N, KSM, R>(wv, fth0, fph0, fth1, fph1, nf, mu, theta_R, it));
            STAMP(25);
            const int rcode = rr & 15;
            it = rr >> 4;
            RELANE();
            vme = lane < NG ? w.V[lane] : R(0.0);
            R lr = R(0.0);
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                const int r = lane + WAVE * q;
                if (r < mo4) {
                    sr[q] = w.ry[r];
                    zl[q] = w.rsig[r];
                    zu[q] = w.rw[r];
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) rv[q][i] = w.V[gen_i(rg[q], i)];
                R o[6];
#pragma unroll
                for (int i = 0; i < 6; ++i) o[i] = w.obs6[6 * roi[q] + i];
                row_trans(rtype[q], rv[q], w.cst[K_GXG], w.cst[K_GYG], ra0[q], ra1[q]);
                cr[q] = row_value(rtype[q], rk[q], rv[q], ra0[q], ra1[q], o, CK);
                const R d1 = sr[q] - cl[q], d2 = cu[q] - sr[q];
                lr += llog(HL(q) ? (HU(q) ? d1 * d2 : d1) : (HU(q) ? d2 : R(1.0)));
                // (kappa_sigma safeguard with the regular barrier parameter, as after every iteration)
                idl[q] = HL(q) ? rcp_nr(d1) : R(0.0);
                idu[q] = HU(q) ? rcp_nr(d2) : R(0.0);
                zl[q] = HL(q) ? fmin(fmax(zl[q], mu * R(1e-10) * idl[q]), R(1e10) * mu * idl[q]) : R(0.0);
                zu[q] = HU(q) ? fmin(fmax(zu[q], mu * R(1e-10) * idu[q]), R(1e10) * mu * idu[q]) : R(0.0);
            }
            lsum_cur = wsum(lr);
            f_cur = obj_sum<N, RPL>(cr, mr4);
            theta_ok = false;
            wave_sync();
            STAMP(24);
            if (rcode == RSW_INFEASIBLE || rcode == RSW_FAILED) {   // Infeasible_Problem_Detected
                status = 2;
                break;
            }
            if (rcode == RSW_MAXITER) break;   // the cap inside the restoration: the final status test below
        }
    }
    for (; it <= max_iter; ++it) {
        // split launch, phase 1: an instance still running at iteration ckpt_it writes its loop state to the next
        // record and stops; phase 2 resumes it on a wave of its own (the long instances no longer share SIMDs).
        // Team-capable build: an instance whose line searches have run ckpt_tr trials (a long search every
        // iteration) stops early and writes a TEAM record, which phase 2 resumes on a workgroup's 4 waves
        // (the cuts run in the lean build, whose count never jumps: a restoration there is cut itself)
        if ((ckpt_it > 0 && it == ckpt_it) || (TM && ckpt_tr > 0 && w.cst[K_NTR] >= R(ckpt_tr))) {
            put_record(TM && !(ckpt_it > 0 && it == ckpt_it), false);
            status = ST_CKPT;
            break;
        }
        // A batch finishes with its slowest instance, and the 4 waves sharing a SIMD compete for issue: waves
        // that have run long get priority, so the critical (high-iteration) instances run closer to their
        // lone-wave latency while the short ones, which have slack, yield.
#ifndef ALIP_NO_SETPRIO
        if (TM && tm < 0)
            ;   // a team member keeps the top priority it resumed with
        else if (it == 8)
            __builtin_amdgcn_s_setprio(1);
        else if (it == 14)
            __builtin_amdgcn_s_setprio(2);
        else if (it == 20)
            __builtin_amdgcn_s_setprio(3);
#endif
        R gl[NT];                                  // J^T y - grad f  (per column, all lanes)
        R jv[JC ? KSM : 1][NT];
        for (;;) {
            RELANE();
            // ---- row layout: generator-form coefficients at V (OBJ rows: grad f_k and its Hessian parts)
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                const int r = lane + WAVE * q;
                R o[6], cf[4], hx[6];
#pragma unroll
                for (int i = 0; i < 6; ++i) o[i] = w.obs6[6 * roi[q] + i];
                row_coef(rtype[q], rk[q], rv[q], ra0[q], ra1[q], o, CK, cf, hx);
                if (r < mo4) {
                    st4(w.rcoef + 4 * r, cf[0], cf[1], cf[2], cf[3]);
                    w.ry[r] = rtype[q] == R_OBJ ? -R(1.0) : zl[q] - zu[q];
                }
                if (rtype[q] == R_VBX) {
                    w.CT[rk[q] + 1] = ra1[q];
                    w.ST[rk[q] + 1] = ra0[q];
                }
                if (rtype[q] == R_OBJ) {
#pragma unroll
                    for (int i = 0; i < 6; ++i) w.hobj[6 * rk[q] + i] = hx[i];
                }
            }
            wave_sync();
            STAMP(0);
            RELANE();
            // ---- J layout: gl = J^T y - grad f (OBJ rows carry y = -1)
#pragma unroll
            for (int T = 0; T < NT; ++T) gl[T] = R(0.0);
            // mo4 == 4 * KSM: every step is a real (possibly padding) row group -> one basic block,
            // all loads in flight together
#pragma unroll
            for (int s = 0; s < KSM; ++s) {
                const int r = 4 * s + g4;
                const uint32_t pk = w.rgen[r];
                struct { R x, y; } ca, cb;
                ld4(w.rcoef + 4 * r, ca.x, ca.y, cb.x, cb.y);
                const R y = w.ry[r];
#pragma unroll
                for (int T = 0; T < NT; ++T) {
                    const int cc = 16 * T + col;
                    const R j = ca.x * G[gen_i(pk, 0) * NCP + cc] + ca.y * G[gen_i(pk, 1) * NCP + cc] +
                                     cb.x * G[gen_i(pk, 2) * NCP + cc] + cb.y * G[gen_i(pk, 3) * NCP + cc];
                    gl[T] += j * y;
                    if constexpr (JC) jv[JC ? s : 0][T] = j;
                }
            }
#pragma unroll
            for (int T = 0; T < NT; ++T) gl[T] = gsum(gl[T]);
            STAMP(1);
            // ---- convergence test (IPOPT scaled overall error) and barrier update
            RELANE();
            R ru = R(0.0);
#pragma unroll
            for (int T = 0; T < NT; ++T)
                if (g4 == 0 && 16 * T + col < n) ru = fmax(ru, fabs(gl[T]));
            // complementarity products w = dl zl, du zu: max |w| and, for every candidate mu of the barrier
            // update, max |w - mu| are attained at the extreme w (|w - mu| is convex in w and fl(w - mu) is
            // monotone in w), so one max and one min replace a reduction per barrier-update trial
            R rcm = R(0.0), nz = R(0.0), whi = -INFINITY, wlo = INFINITY;
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                const R dl = sr[q] - cl[q], du = cu[q] - sr[q];
                if (rtype[q] < R_NONE) rcm = fmax(rcm, fabs(cr[q] - sr[q]));
                nz += fabs(zl[q]) + fabs(zu[q]);
                if (HL(q)) {
                    whi = fmax(whi, dl * zl[q]);
                    wlo = fmin(wlo, dl * zl[q]);
                }
                if (HU(q)) {
                    whi = fmax(whi, du * zu[q]);
                    wlo = fmin(wlo, du * zu[q]);
                }
            }
            // (max(ru)/sd == max(ru/sd): division by sd > 0 and its rounding are monotone, so the stationarity
            // and feasibility maxima share one reduction)
            nz = wsum(nz);
            // (r4: divisions as rcp_div / div100 — a reciprocal and its residual correction instead of the IEEE
            // division sequence)
            const R sd = uni(div100(fmax(R(100.0), rcp_div(nz, w.cst[K_MACT] + n))));
            const R sc = uni(div100(fmax(R(100.0), rcp_div(nz, fmax(R(1.0), w.cst[K_NBL])))));
            const R base_err = wmax(fmax(rcp_div(ru, sd), rcm));
            whi = wmax(whi);
            wlo = wmin(wlo);
            const bool anyw = whi >= wlo;
            const R comp0 = anyw ? fmax(fabs(whi), fabs(wlo)) : R(0.0);
            e0 = uni(fmax(base_err, rcp_div(comp0, sc)));
            // cfg.goal_singular = ABORT: the reference's gradient is NaN at this iterate (cal_dtar_ang_du,
            // MPC_LIP_modi.py:650-655) and IPOPT's Eval_Error ends the solve: Invalid_Number_Detected, iterate kept
            if (rfl(P.goal_abort)) {
                bool at_goal = false;   // an OBJ row's state exactly on the goal
#pragma unroll
                for (int q = 0; q < RPL; ++q) {
                    const R dxg = CK.gxg - rv[q][0], dyg = CK.gyg - rv[q][1];
                    at_goal |= rtype[q] == R_OBJ && dxg * dxg + dyg * dyg == R(0);
                }
                if (__ballot(at_goal) != 0ull) {   // (ends the loop as a factorisation failure does, fail_it)
                    fail_it = it + FAIL_GOAL;
                    it_end = it;
                    break;
                }
            }
            if (e0 <= w.cst[K_TOL]) {
                status = 0;
                break;
            }
            if (it >= it_end) break;
            // IPOPT's floor min(tol, compl_inf_tol) / (barrier_tol_factor + 1 = 11) (MonotoneMuUpdate): tol / 11 for
            // every tol <= compl_inf_tol = 1e-4 (the fp32 defaults above it keep their own tol / 11)
            const R mu_min = w.cst[K_TOL] / R(11.0);
            const R mu_prev = mu;
            for (int t = 0; t < 8; ++t) {
                const R cm = anyw ? fmax(fabs(whi - mu), fabs(wlo - mu)) : R(0.0);
                if (fmax(base_err, rcp_div(cm, sc)) <= R(10.0) * mu && mu > mu_min)
                    mu = uni(fmax(mu_min, fmin(R(0.2) * mu, mu * sqrt(mu))));
                else
                    break;
            }
            if (mu != mu_prev) nf = 0;
            break;
        }
        STAMP(2);
        if (status == 0 || it >= it_end) break;
        const R tau = uni(fmax(R(0.99), R(1.0) - mu));

        // ---- Sigma, rhs weights, Hessian blocks
        RELANE();
        R rcv[RPL];
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int r = lane + WAVE * q;
            const R sg = zl[q] * idl[q] + zu[q] * idu[q];
            rcv[q] = rtype[q] < R_NONE ? cr[q] - sr[q] : R(0.0);
            R wr = mu * idl[q] - mu * idu[q] - sg * rcv[q];
            wr = rtype[q] == R_OBJ ? -R(1.0) : wr;
            if (r < mo4) {
                w.rsig[r] = sg;
                w.rw[r] = wr;
            }
        }
        RELANE();
#ifndef ALIP_HESS_SERIAL
        if constexpr (16 * (N + 1) <= WAVE)
            hess_blocks_lanes<N, R>(w, lane, rps, nobs, modi);
        else
#endif
            hess_blocks<N, R>(w, lane, rps, nobs, modi);
        wave_sync();
        STAMP(3);
        // ---- K = J^T Sigma J + G^T S G by f64 MFMA (two accumulator chains), rhs = J^T w - grad f
        R rhsc[NT];
        RELANE();
        {
            constexpr int NA = NT * (NT + 1) / 2;
            typename Mfma<R>::acc acc[2][NA];
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int i = 0; i < NA; ++i) acc[h][i] = typename Mfma<R>::acc{R(0), R(0), R(0), R(0)};
            R pw[NT];
#pragma unroll
            for (int T = 0; T < NT; ++T) pw[T] = R(0.0);
#pragma unroll
            for (int s = 0; s < KSM; ++s) {
                const int r = 4 * s + g4;
                const R sg = w.rsig[r], wr = w.rw[r];   // padding / OBJ rows: sigma = 0
                R j[NT];
                if constexpr (JC) {
#pragma unroll
                    for (int T = 0; T < NT; ++T) j[T] = jv[JC ? s : 0][T];
                } else {
                    const uint32_t pk = w.rgen[r];
                    struct { R x, y; } ca, cb;
                    ld4(w.rcoef + 4 * r, ca.x, ca.y, cb.x, cb.y);
#pragma unroll
                    for (int T = 0; T < NT; ++T) {
                        const int cc = 16 * T + col;
                        j[T] = ca.x * G[gen_i(pk, 0) * NCP + cc] + ca.y * G[gen_i(pk, 1) * NCP + cc] +
                               cb.x * G[gen_i(pk, 2) * NCP + cc] + cb.y * G[gen_i(pk, 3) * NCP + cc];
                    }
                }
#pragma unroll
                for (int T = 0; T < NT; ++T) pw[T] += j[T] * wr;
                auto* a = acc[s & 1];
                a[0] = Mfma<R>::run(j[0], sg * j[0], a[0]);
                if constexpr (NT == 2) {
                    a[1] = Mfma<R>::run(j[0], sg * j[1], a[1]);
                    a[2] = Mfma<R>::run(j[1], sg * j[1], a[2]);
                }
            }
#pragma unroll
            for (int s = 1; s < NG / 4; ++s) {
                const int t = 4 * s + g4;
                const int kb = t >> 3, c = t & 7;
                const R* Srow = w.S + 64 * kb + 8 * c;
                const R* Gb = G + 8 * kb * NCP;
                R gv[NT], sgv[NT];
                // S rows 0..3 (even s: t & 7 = g4) have nonzeros in columns {0, 1, 4, 5, 6} only, rows 4..7 in {0..6}
                // (hess_blocks' pattern; the rest of S stays zero): the zero products are skipped (+0 terms, the same
                // sums)
#ifdef ALIP_S_DENSE   // dev A/B: every column
                const unsigned SCOLS = 0xFFu;
#else
                const unsigned SCOLS = (s & 1) ? 0x7Fu : 0x73u;   // (s is unrolled: a constant per step)
#endif
#pragma unroll
                for (int T = 0; T < NT; ++T) {
                    gv[T] = G[t * NCP + 16 * T + col];
                    R a = R(0.0);
#pragma unroll
                    for (int c2 = 0; c2 < 8; ++c2)
                        if ((SCOLS >> c2) & 1u) a += Srow[c2] * Gb[c2 * NCP + 16 * T + col];
                    sgv[T] = a;
                }
                auto* a = acc[s & 1];
                a[0] = Mfma<R>::run(gv[0], sgv[0], a[0]);
                if constexpr (NT == 2) {
                    a[1] = Mfma<R>::run(gv[0], sgv[1], a[1]);
                    a[2] = Mfma<R>::run(gv[1], sgv[1], a[2]);
                }
            }
#pragma unroll
            for (int T = 0; T < NT; ++T) rhsc[T] = gsum(pw[T]);
            // C/D layout (Mfma<R>::row): f64 lane holds D[g4 + 4*i][col], f32 D[4*g4 + i][col], i = 0..3
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = Mfma<R>::row(g4, i);
                w.K[row * KLD + col] = acc[0][0][i] + acc[1][0][i];
                if constexpr (NT == 2) {
                    const R k1 = acc[0][1][i] + acc[1][1][i];
                    w.K[row * KLD + 16 + col] = k1;
                    w.K[(16 + col) * KLD + row] = k1;
                    w.K[(16 + row) * KLD + 16 + col] = acc[0][2][i] + acc[1][2][i];
                }
            }
        }
        wave_sync();
        STAMP(4);
        // ---- factor with inertia correction, solve for dp.  n <= 9 (N <= 3): Gauss-Jordan on [K + dw I | rhs]
        // in LDS (gj_lds); larger n: register Cholesky (chol_rows) + two triangular sweeps, which measured
        // faster there (GJ work grows as n * ceil(n (n+1) / 64) element updates)
        RELANE();
        R xv;
        bool fact_ok = true;   // false: regularisation exhausted (IPOPT's Error_In_Step_Computation)
        {
            R rhs_l = R(0.0);
#pragma unroll
            for (int T = 0; T < NT; ++T) rhs_l = (lane < n && (lane >> 4) == T) ? rhsc[T] : rhs_l;
            if constexpr (GJ && GJ_REGS) {
                // [K | rhs] rows in registers (K stays in w.K for inertia-correction retries)
                R a[n + 1];
                auto fill = [&](R dw) {
#pragma unroll
                    for (int j = 0; j < n; ++j) a[j] = (lane < n ? w.K[lane * KLD + j] : R(0.0)) + (lane == j ? dw : R(0.0));
                    a[n] = rhs_l + R(0.0);
                };
                fill(R(0));
                if (!gj_regs<n>(a, lane)) {
                    R dw = dw_last == R(0.0) ? R(1e-4) : fmax(R(1e-20), dw_last / R(3.0));
                    for (;;) {
                        fill(dw);
                        if (gj_regs<n>(a, lane)) break;
                        dw *= dw_last == R(0.0) ? R(100.0) : R(8.0);
                        if (dw > R(sizeof(R) == 8 ? 1e40 : 1e30)) {   // (not IPOPT's 1e20)
                            fact_ok = false;
                            break;
                        }
                    }
                    dw_last = uni(dw);
                }
                xv = lane < n ? a[n] : R(0.0);
            } else if constexpr (GJ) {
                // [K | rhs] stays in w.K (the original, for inertia-correction retries); the elimination runs on
                // a copy in the S-block buffer, which is dead once K is built and is re-zeroed after dV below
                if (lane < n) w.K[lane * KLD + n] = rhs_l;
                wave_sync();
                gj_fill<n, KLD, GJLD>(w.K, w.S, lane, R(0));
                wave_sync();
                if (!gj_lds<n, GJLD>(w.S, lane)) {
                    R dw = dw_last == R(0.0) ? R(1e-4) : fmax(R(1e-20), dw_last / R(3.0));
                    for (;;) {
                        gj_fill<n, KLD, GJLD>(w.K, w.S, lane, dw);
                        wave_sync();
                        if (gj_lds<n, GJLD>(w.S, lane)) break;
                        dw *= dw_last == R(0.0) ? R(100.0) : R(8.0);
                        if (dw > R(sizeof(R) == 8 ? 1e40 : 1e30)) {   // (not IPOPT's 1e20)
                            fact_ok = false;
                            break;
                        }
                    }
                    dw_last = uni(dw);
                }
                xv = lane < n ? w.S[lane * GJLD + n] : R(0.0);
            } else {
                R a[n];
                R myidg = R(1.0);
#pragma unroll
                for (int j = 0; j < n; ++j) a[j] = lane < n ? w.K[lane * KLD + j] : (lane == j ? R(1.0) : R(0.0));
                if (!chol_rows<n>(a, myidg, lane)) {
                    R dw = dw_last == R(0.0) ? R(1e-4) : fmax(R(1e-20), dw_last / R(3.0));
                    for (;;) {
#pragma unroll
                        for (int j = 0; j < n; ++j)
                            a[j] = (lane < n ? w.K[lane * KLD + j] : (lane == j ? R(1.0) : R(0.0))) +
                                   (lane == j ? dw : R(0.0));
                        if (chol_rows<n>(a, myidg, lane)) break;
                        dw *= dw_last == R(0.0) ? R(100.0) : R(8.0);
                        if (dw > R(sizeof(R) == 8 ? 1e40 : 1e30)) {   // (not IPOPT's 1e20)
                            fact_ok = false;
                            break;
                        }
                    }
                    dw_last = uni(dw);
                }
                // forward: L y = rhs
                R acc = R(0.0), yv = R(0.0);
#pragma unroll
                for (int k = 0; k < n; ++k) {
                    const R yk = bcast((rhs_l - acc) * myidg, k);
                    yv = lane == k ? yk : yv;
                    acc += lane > k ? a[k] * yk : R(0.0);
                }
                // transpose L through LDS for the backward sweep
                wave_sync();
                if (lane < n) {
#pragma unroll
                    for (int j = 0; j < n; ++j) w.K[lane * KLD + j] = j <= lane ? a[j] : R(0.0);
                }
                wave_sync();
                acc = R(0.0);
                xv = R(0.0);
#pragma unroll
                for (int i = n - 1; i >= 0; --i) {
                    const R xi = bcast((yv - acc) * myidg, i);
                    xv = lane == i ? xi : xv;
                    acc += lane < i ? w.K[i * KLD + (lane & 31)] * xi : R(0.0);
                }
            }
        }
        STAMP(5);
        // ---- dV = G dp (lane t), rows pick up their 4 entries; GJ: dp is column n of the eliminated system
        // in LDS (broadcast reads), Cholesky: dp is in lane registers (readlane)
        RELANE();
        {
            R v = R(0.0);
#pragma unroll
            for (int j = 0; j < n; ++j)
                v += G[(lane < NG ? lane : 0) * NCP + j] * (GJ && !GJ_REGS ? w.S[j * GJLD + n] : bcast(xv, j));
            // a factorisation the regularisation could not rescue: zero step (the iterate stays), and the
            // solve ends at the next iteration's test with status -3 (no extra loop exit here: an exit
            // edge in mid-iteration lengthens live ranges and costs spills)
            dvme = lane < NG && fact_ok ? v : R(0.0);
            if (lane < NG) w.dV[lane] = dvme;
        }
        wave_sync();
        if constexpr (GJ && !GJ_REGS) gj_zero<n, GJLD>(w.S, lane);   // hess_blocks writes only the nonzero pattern of S
        if (!fact_ok && fail_it < 0) {
            fail_it = it;
            it_end = it + 1;
        }
        // ---- slack / multiplier steps, fraction to boundary
        RELANE();
        R dS[RPL], dZl[RPL], dZu[RPL];
        R ap = R(1.0), az = R(1.0), theta = R(0.0), sl = R(0.0), jdv[RPL];
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int r = lane + WAVE * q;
#pragma unroll
            for (int i = 0; i < 4; ++i) rdv[q][i] = w.dV[gen_i(rg[q], i)];
            R jd = R(0.0);
            if (r < mo4) {
                struct { R x, y; } ca, cb;
                ld4(w.rcoef + 4 * r, ca.x, ca.y, cb.x, cb.y);
                jd = ca.x * rdv[q][0] + ca.y * rdv[q][1] + cb.x * rdv[q][2] + cb.y * rdv[q][3];
            }
            jdv[q] = jd;
            dS[q] = rtype[q] < R_NONE ? jd + rcv[q] : R(0.0);
            dZl[q] = HL(q) ? mu * idl[q] - zl[q] - zl[q] * idl[q] * dS[q] : R(0.0);
            dZu[q] = HU(q) ? mu * idu[q] - zu[q] + zu[q] * idu[q] * dS[q] : R(0.0);
            const R dl = sr[q] - cl[q], du = cu[q] - sr[q];
            const R ids = rcp_nr(dS[q]);
            if (HL(q) && dS[q] < 0) ap = fmin(ap, -tau * dl * ids);
            if (HU(q) && dS[q] > 0) ap = fmin(ap, tau * du * ids);
            if (HL(q) && dZl[q] < 0) az = fmin(az, -tau * zl[q] * rcp_nr(dZl[q]));
            if (HU(q) && dZu[q] < 0) az = fmin(az, -tau * zu[q] * rcp_nr(dZu[q]));
            theta += fabs(rcv[q]);
            sl += (HL(q) ? dS[q] * idl[q] : R(0.0)) - (HU(q) ? dS[q] * idu[q] : R(0.0));
        }
        ap = wmin(ap);
        az = wmin(az);
        // theta = sum |c - s| at the current point: the accepted trial's value (same operations, same order)
        // unless the point came from the initial set-up or a restoration reset
        theta = theta_ok ? theta_c : wsum(theta);
        const R gdv = obj_sum<N, RPL>(jdv, mr4);
        sl = wsum(sl);
        const R phi = uni(f_cur - mu * lsum_cur);
        const R gphi = uni(gdv - mu * sl);
        // switching condition a (-gphi)^s_phi > theta^s_theta in log space: log a + s_phi llog(-gphi) >
        // s_theta log theta (two logs per iteration instead of two pow per trial)
        const R lsw = uni(gphi < 0 ? sth * llog(theta) - sph * llog(-gphi) : R(0.0));
        R amin;
        if (gphi < 0) {
            amin = fmin(gth, gph * theta / -gphi);
            if (theta <= w.cst[K_THMIN]) amin = fmin(amin, exp(lsw));
        } else {
            amin = gth;
        }
        // floor 2^-60 where the formula gives 0 (theta = 0 exactly, DESIGN.md §2 item 8: the trials a = ap 2^-j would
        // never fall below it); a positive amin, however small, is IPOPT's own
        amin *= gal;
        amin = uni(amin > R(0) ? amin : R(8.673617379884035e-19));
        STAMP(6);
        // ---- filter line search on trial points V + a dV (row registers only)
        // Trial j is a_j = ap 2^-j (and log a_j by the same sequential subtractions); the search takes the first
        // acceptable trial with a_j >= amin.  A team (4 waves in lockstep on one instance, team-capable build)
        // evaluates trials J + member in one round, exchanges accept flags through LDS, and every member other than
        // the first accepting one re-evaluates that trial: the same trials, the same arithmetic, the same choice as one
        // wave.
        R a = ap;
        R la = uni(llog(ap));   // log a, tracked exactly through the halvings
        bool accepted = false, ftype = false;
        R ctr[RPL], ta0[RPL], ta1[RPL];
        R ft = R(0.0), lgt = R(0.0), tht_acc = R(0.0);
        bool redo = false;   // team: this pass re-evaluates the winning trial (a, la already advanced to it)
        for (;;) {
            R am = a, lam = la;   // this member's trial
            if (!(TM && redo))
                for (int t = 0; t < -1 - tm; ++t) {
                    am = uni(am * R(0.5));
                    lam = uni(lam - R(M_LN2));
                }
            const bool valid = am >= amin;
            bool acc_m = false, fty_m = false;
            if (valid) {
                WSTAMP_TRIAL;
                RELANE();
                R tht = R(0.0);
                ft = R(0.0);
                lgt = R(0.0);
                bool bad = false;
#pragma unroll
                for (int q = 0; q < RPL; ++q) {
                    // the trial point is rebuilt from (rv, rdv, a) where needed (on acceptance, the same fma)
                    R vt[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) vt[i] = fma(am, rdv[q][i], rv[q][i]);
                    R o[6];
#pragma unroll
                    for (int i = 0; i < 6; ++i) o[i] = w.obs6[6 * roi[q] + i];
                    row_trans(rtype[q], vt, w.cst[K_GXG], w.cst[K_GYG], ta0[q], ta1[q]);
                    ctr[q] = row_value(rtype[q], rk[q], vt, ta0[q], ta1[q], o, CK);
                    const R st = sr[q] + am * dS[q];
                    if (rtype[q] < R_NONE) tht += fabs(ctr[q] - st);

                    const R d1 = st - cl[q], d2 = cu[q] - st;
                    if (HL(q) && !(d1 > 0)) bad = true;
                    if (HU(q) && !(d2 > 0)) bad = true;
                    // one log per lane (the bound pattern selects its argument; log 1 = 0): the three-way select of
                    // logs had compiled to three log evaluations per trial
                    lgt += llog(HL(q) ? (HU(q) ? d1 * d2 : d1) : (HU(q) ? d2 : R(1.0)));
                }
                tht = wsum(tht);
                ft = obj_sum<N, RPL>(ctr, mr4);
                lgt = wsum(lgt);
                const bool anybad = __ballot(bad) != 0ull;
                const R pht = anybad ? INFINITY : ft - mu * lgt;
                bool ok = isfinite(pht) && tht < w.cst[K_THMAX];
                if (ok) {
                    const bool b0 = lane < nf && !(tht < fth0 || pht < fph0);
                    const bool b1 = lane + WAVE < nf && !(tht < fth1 || pht < fph1);
                    ok = __ballot(b0 || b1) == 0ull;
                }
                if (ok) {
                    const bool switching = gphi < 0 && lam > lsw;
                    if (switching && theta <= w.cst[K_THMIN]) {
                        if (pht <= phi + eta * am * gphi) {
                            acc_m = true;
                            fty_m = true;
                        }
                    } else if (tht <= (1 - gth) * theta || pht <= phi - gph * theta) {
                        acc_m = true;
                        fty_m = false;
                    }
                }
                tht_acc = tht;
            }
            if (TM && redo) {   // the winner's trial values are this member's now
                accepted = true;
                break;
            }
            if (!TM || tm >= 0) {
                if (!valid) break;
                if (acc_m) {
                    accepted = true;
                    ftype = fty_m;
                    break;
                }
                a = uni(a * R(0.5));
                la = uni(la - R(M_LN2));
                continue;
            }
            // team round: member m's accept flag for round parity p sits in m's own workspace (Vt[p]: prologue
            // scratch, free afterwards); a member's next write to a parity follows the barrier that every reader of
            // the previous one passes first
            if constexpr (!TM) break;
            {
                const int me = -1 - tm;
                const int wss = wss_elems<N, R>(rfl(P.nc_max), rfl(P.ne_max), rfl(P.mr4), rfl(P.mo4));
                const int par = w.cst[K_XR] != R(0.0) ? 1 : 0;
                if (lane == 0) {
                    w.Vt[par] = R(valid ? (acc_m ? (fty_m ? 3 : 2) : 1) : 0);
                    w.cst[K_XR] = R(1 - par);
                }
                __syncthreads();
                const R* vt0 = w.Vt - me * wss;   // member 0's flags
                // first member whose trial did not end in a rejection, and its flag (the members' flags read together)
                int fl[TEAM_WAVES];
#pragma unroll
                for (int m = 0; m < TEAM_WAVES; ++m) fl[m] = (int)vt0[m * wss + par];
                int wn = TEAM_WAVES, fw = 0;
#pragma unroll
                for (int m = TEAM_WAVES - 1; m >= 0; --m) {
                    wn = fl[m] != 1 ? m : wn;
                    fw = fl[m] != 1 ? fl[m] : fw;
                }
                wn = rfl(wn);
                fw = rfl(fw);
                for (int t = 0; t < wn; ++t) {   // a, la of trial J + wn (J + TEAM_WAVES when all rejected)
                    a = uni(a * R(0.5));
                    la = uni(la - R(M_LN2));
                }
                if (wn == TEAM_WAVES) continue;
                if (fw == 0) break;   // trial J + wn is below amin: no acceptable trial
                ftype = fw == 3;
                if constexpr (TEAM_HANDOVER<N, RPL>) {
                    // hand-over: the winner's trial values (row values and transcendentals, f, the log sum, theta)
                    // go to the others through the winner's KKT area, dead until the next iteration's K products; a
                    // second barrier orders the reads before that overwrite
                    R* hv = w.K + (wn - me) * wss;
                    if (wn == me) {
#pragma unroll
                        for (int q = 0; q < RPL; ++q) {
                            hv[(3 * q) * WAVE + lane] = ctr[q];
                            hv[(3 * q + 1) * WAVE + lane] = ta0[q];
                            hv[(3 * q + 2) * WAVE + lane] = ta1[q];
                        }
                        if (lane == 0) {
                            hv[3 * RPL * WAVE] = ft;
                            hv[3 * RPL * WAVE + 1] = lgt;
                            hv[3 * RPL * WAVE + 2] = tht_acc;
                        }
                    }
                    __syncthreads();
                    if (wn != me) {
#pragma unroll
                        for (int q = 0; q < RPL; ++q) {
                            ctr[q] = hv[(3 * q) * WAVE + lane];
                            ta0[q] = hv[(3 * q + 1) * WAVE + lane];
                            ta1[q] = hv[(3 * q + 2) * WAVE + lane];
                        }
                        ft = uni(hv[3 * RPL * WAVE]);
                        lgt = uni(hv[3 * RPL * WAVE + 1]);
                        tht_acc = uni(hv[3 * RPL * WAVE + 2]);
                    }
                    __syncthreads();
                    accepted = true;
                    break;
                }
                if (wn == me) {
                    accepted = true;
                    break;
                }
                redo = true;
            }
        }
        STAMP(7);
        // trials of this search (a = ap 2^-j: j + 1 evaluated when trial j was taken, j when a fell below amin)
        if (TM && ckpt_tr > 0 && lane == 0)
            w.cst[K_NTR] += R(fexp2(ap) - fexp2(a) + (accepted ? 1 : 0));
        RELANE();
        if (accepted) {
            if (!ftype && nf < FILTER_CAP) {
                const R fvt = (1 - gth) * theta, fvp = phi - gph * theta;
                if ((nf & (WAVE - 1)) == lane) {
                    if (nf < WAVE) {
                        fth0 = fvt;
                        fph0 = fvp;
                    } else {
                        fth1 = fvt;
                        fph1 = fvp;
                    }
                }
                nf++;
            }
            vme = fma(a, dvme, vme);
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
#pragma unroll
                for (int i = 0; i < 4; ++i) rv[q][i] = fma(a, rdv[q][i], rv[q][i]);
                ra0[q] = ta0[q];
                ra1[q] = ta1[q];
                sr[q] += a * dS[q];
                cr[q] = ctr[q];
            }
            f_cur = ft;
            lsum_cur = lgt;
            theta_c = tht_acc;
            theta_ok = true;
        } else if (rfl(P.resto_ipopt)) {
            // cfg.restoration = IPOPT: the failed point (this iteration counts) goes to the restoration phase after
            // this loop
            status = ST_RESTO;
            it++;
            break;
        } else {
            theta_ok = false;
            // restoration substitute: shortest tried step, slacks reset onto c(u), filter reset
            a = uni(fmax(a, amin));
            vme = fma(a, dvme, vme);
            R fr = R(0.0), lr = R(0.0);
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
#pragma unroll
                for (int i = 0; i < 4; ++i) rv[q][i] = fma(a, rdv[q][i], rv[q][i]);
                R o[6];
#pragma unroll
                for (int i = 0; i < 6; ++i) o[i] = w.obs6[6 * roi[q] + i];
                row_trans(rtype[q], rv[q], w.cst[K_GXG], w.cst[K_GYG], ra0[q], ra1[q]);
                cr[q] = row_value(rtype[q], rk[q], rv[q], ra0[q], ra1[q], o, CK);
                R v = cr[q];
                const R pl = HL(q) ? fmin(R(1e-2) * fmax(R(1.0), fabs(cl[q])), R(1e-2) * (cu[q] - cl[q])) : R(0.0);
                const R pu = HU(q) ? fmin(R(1e-2) * fmax(R(1.0), fabs(cu[q])), R(1e-2) * (cu[q] - cl[q])) : R(0.0);
                if (HL(q) && HU(q))
                    v = fmin(fmax(v, cl[q] + pl), cu[q] - pu);
                else if (HL(q))
                    v = fmax(v, cl[q] + pl);
                else if (HU(q))
                    v = fmin(v, cu[q] - pu);
                sr[q] = rtype[q] < R_NONE ? v : R(0.0);
                const R d1 = sr[q] - cl[q], d2 = cu[q] - sr[q];
                lr += llog(HL(q) ? (HU(q) ? d1 * d2 : d1) : (HU(q) ? d2 : R(1.0)));

            }
            lr = wsum(lr);
            fr = obj_sum<N, RPL>(cr, mr4);
            f_cur = fr;
            lsum_cur = lr;
            nf = 0;
            // infeasibility detection (stands in for IPOPT's failed restoration phase)
            n_rest++;
            R viol = R(0.0);
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                const int r = lane + WAVE * q;
                if (r < mr4 && rtype[q] < R_NONE) {
                    if (HL(q)) viol = fmax(viol, w.rclo[r] - cr[q]);
                    if (HU(q)) viol = fmax(viol, cr[q] - w.rcuo[r]);
                }
            }
            viol = wmax(viol);
            if (n_rest >= REST_FAIL && viol > R(1e-4)) {
                if (lane < NG) w.V[lane] = vme;
                status = 2;
                it++;
                break;
            }
        }
        if (lane < NG) w.V[lane] = vme;
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            zl[q] += az * dZl[q];
            zu[q] += az * dZu[q];
            const R d1 = sr[q] - cl[q], d2 = cu[q] - sr[q];
            idl[q] = HL(q) ? rcp_nr(d1) : R(0.0);
            idu[q] = HU(q) ? rcp_nr(d2) : R(0.0);
            zl[q] = HL(q) ? fmin(fmax(zl[q], mu * R(1e-10) * idl[q]), R(1e10) * mu * idl[q]) : R(0.0);
            zu[q] = HU(q) ? fmin(fmax(zu[q], mu * R(1e-10) * idu[q]), R(1e10) * mu * idu[q]) : R(0.0);
        }
        wave_sync();
        STAMP(9);
    }
    if (status != ST_RESTO) break;
    if constexpr (sizeof(R) == 4) {   // fp32: the fp64 wave program solves this instance from its start (the
        // stream's hand-off list, P.redo; launch() runs it after this launch).  The fp32 restoration phase took other
        // paths than the oracle's on the tolerance edges, and fp32's one lean build keeps every launch form
        // bit-identical.
        if (!P.redo) {   // (the host always provides the list; no write without one)
            status = 2;
            break;
        }
        if (lane == 0) {
            const uint32_t k = atomicAdd(P.redo, 1u);
            P.redo[1 + k] = (uint32_t)b;
        }
        status = ST_CKPT;
        break;
    }
    // the failed point (this iteration counted) enters the filter — IPOPT's augmented filter, with the point's
    // violation (the same sum as the iteration's theta) and barrier function — then the restoration phase from it
    ++n_rest;
    {
        RELANE();
        R th = R(0.0);
#pragma unroll
        for (int q = 0; q < RPL; ++q)
            if (rtype[q] < R_NONE) th += fabs(cr[q] - sr[q]);
        theta_R = theta_ok ? theta_c : wsum(th);
        phi_R = uni(f_cur - mu * lsum_cur);
    }
    if (nf < FILTER_CAP) {
        const R fvt = (1 - gth) * theta_R, fvp = phi_R - gph * theta_R;
        if ((nf & (WAVE - 1)) == lane) {
            if (nf < WAVE) {
                fth0 = fvt;
                fph0 = fvp;
            } else {
                fth1 = fvt;
                fph1 = fvp;
            }
        }
        nf++;
    }
    theta_ok = false;
    status = -1;
    if constexpr (!RS) {   // the lean build (phase 1 of a split launch): phase 2's RS build runs the phase
        put_record(false, true);
        status = ST_CKPT;
        break;
    }
    rpend = true;
    }
    STAMP(8);
    STAMP_FLUSH;
    if (status == ST_CKPT) {   // phase 2 of the split launch finishes this instance
        WSTAMP_WRITE(b, it, n_rest);
        return;
    }
    if (fail_it >= FAIL_GOAL) {   // cfg.goal_singular = ABORT: Invalid_Number_Detected at this iterate
        status = -13;
        it = fail_it - FAIL_GOAL;
    } else if (fail_it >= 0) {   // the last iterate, as IPOPT returns it with Error_In_Step_Computation
        status = -3;
        it = fail_it;
    }
    // ---- status + outputs (violation measured on the reference's exact |.|)
    wave_sync();
    RELANE();
    if (status != 0 && status != 2 && status != -3 && status != -13) {
        R viol = R(0.0);
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int r = lane + WAVE * q;
            R o[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) o[i] = w.obs6[6 * roi[q] + i];
            const R c = row_value(rtype[q], rk[q], rv[q], ra0[q], ra1[q], o, CK);
            if (r < mr4 && rtype[q] < R_NONE) {
                if (HL(q)) viol = fmax(viol, w.rclo[r] - c);
                if (HU(q)) viol = fmax(viol, c - w.rcuo[r]);
            }
        }
        viol = wmax(viol);
        if (e0 <= w.cst[K_ACCTOL])
            status = 1;
        else if (viol > R(1e-4))
            status = 2;
    }
    if (TM && tm < -1) return;   // team members 1..3 computed the same outputs as member 0 (tm = -1)
    WSTAMP_WRITE(rec >= 0 ? P.B + rec : b, it, n_rest);   // (diagnostic build: phase-2 records after the batch's)
    // canonical u: u_k = x_{k+1} (W u_k = p_k since W B = I) — the reference's "desired next state"
    if (lane < 5 * N) P.u_out[(size_t)b * 5 * N + lane] = w.V[gx(lane / 5 + 1, lane % 5)];
    if (P.foot_out && lane < 3) P.foot_out[3 * b + lane] = w.V[gp(0, lane)];
    if (P.x_pred && lane < 5 * N) P.x_pred[(size_t)b * 5 * N + lane] = w.V[gx(lane / 5 + 1, lane % 5)];
    if (lane == 0) {
        if (P.status) P.status[b] = status;
        if (P.iters) P.iters[b] = it;
    }
#undef RELANE
#undef CK
#undef HL
#undef HU
}

// work-queue instance source of a persistent launch: counters q[0] (next instance) and q[1] (waves that
// found the queue empty); the last wave out resets both, so the next launch on the stream starts at 0
__device__ __forceinline__ long long next_instance(uint32_t* q)
{
    uint32_t v = 0;
    if (lane_id() == 0) v = atomicAdd(q, 1u);
    return (long long)__builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ void queue_exit(uint32_t* q)
{
    __threadfence();
    if (lane_id() == 0 && atomicAdd(q + 1, 1u) == gridDim.x * WAVES_PER_BLOCK - 1) {
        atomicExch(q, 0u);
        atomicExch(q + 1, 0u);
    }
}

#ifndef ALIP_WAVES_RPL1
#define ALIP_WAVES_RPL1 4
#endif
#ifndef ALIP_WAVES_RPL2
#define ALIP_WAVES_RPL2 2
#endif
// waves per SIMD the register budget is sized for (512 / waves VGPRs per lane).  One row group per lane
// (RPL = 1): 4 waves, 128 VGPRs, a few spilled values.  Two row groups (RPL = 2, N >= 4 or many
// obstacles): the row state alone is ~110 VGPRs, and at 128 VGPRs it spilled 400 B/lane; 2 waves with
// 256 VGPRs spill nothing and measured +48 % on cfg3 (profiles/r1f/ab_occupancy.log)
// fp32, one row group: 93-103 VGPRs at 4 waves; 7 waves (72 VGPRs, some spills in the queue kernel)
// measured best on cfg5: 4 -> 5 -> 6 -> 7 -> 8 waves = 21.0 / 21.9 / 22.7 / 23.1 / 22.1 M solves/s
// (profiles/r1f/ab_fp32_occupancy.log)
#ifndef ALIP_WAVES_F32
#define ALIP_WAVES_F32 7
#endif
#ifndef ALIP_WAVES_RS
#define ALIP_WAVES_RS 2
#endif
template <int KSM, class R, bool RSW = false>
constexpr int solve_waves()
{
    // RSW: the restoration-capable builds (fp64; split phase 2, one-phase launches, the work queue and the hand-off
    // queue) take the registers of 2 waves per SIMD instead of spilling: the phase-2 instances run on lone waves, and
    // at 4 waves the work-queue build spilled 520 B/lane (r6)
    return 4 * KSM > WAVE ? ALIP_WAVES_RPL2
                          : (RSW ? (sizeof(R) == 4 ? 4 : ALIP_WAVES_RS) : (sizeof(R) == 4 ? ALIP_WAVES_F32 : ALIP_WAVES_RPL1));
}

// Launch forms of one solve program.  A batch larger than the resident slots runs the persistent work queue:
// a grid of the resident workgroups whose waves take instances with one atomicAdd each, so a wave that
// finishes a short solve takes the next instance at once instead of idling until its workgroup's longest
// solve ends.  A batch that fits the slots (B <= alipmpc_solve_slots, cfg2) needs no queue: one instance per
// wave, no instance loop — the loop-carried values of the persistent form cost registers (scratch 76 -> 44
// B/lane) and 11 % of the cfg2 launch (tools/ab_solve.py, profiles/r2).  Both forms inline the same
// solve_one and produce the same bits for an instance (test_work_queue_batch_independence solves a batch
// above the slots whole and in half-slot chunks and compares status, iters, u, foot, x_pred exactly), so an
// instance's result does not depend on its batch or on the device's slot count.
template <int N, int KSM, class R, bool ONE, bool TM = false, bool RS = false>
__global__ __launch_bounds__(WAVE * (TM ? TEAM_WAVES : WAVES_PER_BLOCK), (solve_waves<KSM, R, RS>())) void solve_kernel(KP Pv)
{
    constexpr int WPB = TM ? TEAM_WAVES : WAVES_PER_BLOCK;   // waves per workgroup (team-capable: the team size)
    using D = Dim<N>;
    constexpr int NCP = D::NCP;
    constexpr int NG = D::NG;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    KP* Ps = reinterpret_cast<KP*>(smem);
    R* G = reinterpret_cast<R*>(smem + KP_DOUBLES);
    // (r4: no LDS copy of E — the prologue reads it from global memory once per instance)
    R* wsb = G + NG * NCP;
    if (threadIdx.x == 0) *Ps = Pv;
    for (int i = threadIdx.x; i < NG * NCP; i += blockDim.x) G[i] = Pv.G[i];
    __syncthreads();
    const KP& P = *Ps;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);   // wave-uniform (SGPR)
    // slot k of the launch (wave k, or the k-th queue ticket) solves instance order[k] (identity without an order):
    // the per-instance arithmetic does not depend on the slot, only when and where the instance runs
    if constexpr (ONE) {
        // split phase 2 of the team-capable build: workgroups [0, Pv.team) resume team records (the workgroup's WPB
        // waves in lockstep on one instance), the rest single records one wave each, then any team records beyond
        // Pv.team
        const long long nteamwg = TM && Pv.resume ? (long long)Pv.team : 0;
        const bool team = (long long)blockIdx.x < nteamwg;
        const long long k = team ? (long long)blockIdx.x : ((long long)blockIdx.x - nteamwg) * WPB + wv;
        long long b = -1, rec = -1;   // one inlined solve_one for every form (the code is large)
        if (Pv.resume) {   // split launch, phase 2
            const long long made = TM ? (long long)__builtin_amdgcn_readfirstlane(Pv.cont[CONT_TEAM]) : 0;
            if (team) {
                if (k < made) rec = Pv.B - 1 - k;
            } else {
                const long long cnt = (long long)__builtin_amdgcn_readfirstlane(Pv.cont[CONT_SINGLE]);
                if (k < cnt)
                    rec = k;
                else if (k - cnt + nteamwg < made)
                    rec = Pv.B - 1 - (k - cnt + nteamwg);
            }
            if (rec >= 0) b = (long long)__builtin_amdgcn_readfirstlane(Pv.cont[cont_hdr(Pv.B) + rec]);
        } else if (k < Pv.B) {
            b = Pv.order ? (long long)__builtin_amdgcn_readfirstlane(Pv.order[k]) : k;
            if (Pv.active && !Pv.active[b]) b = -1;
        }
        b = __builtin_amdgcn_readfirstlane((int)b);
        rec = __builtin_amdgcn_readfirstlane((int)rec);
        // (one call site: the team solves run the very machine code of the single ones — two inlined copies had
        // rounded differently)
        if (b >= 0) solve_one<N, KSM, R, false, TM, RS>(P, G, wsb, wv, b, rec, team ? -1 - wv : 0);
    } else {
        uint32_t* const q = Pv.queue;
        // (a hand-off launch: the count of the list it solves was written on the device by the launch before it)
        const long long Bq = Pv.bcount ? std::min(Pv.B, (long long)__builtin_amdgcn_readfirstlane((int)*Pv.bcount)) : Pv.B;
        for (long long k = next_instance(q); k < Bq; k = next_instance(q)) {
            const long long b = Pv.order ? (long long)__builtin_amdgcn_readfirstlane(Pv.order[k]) : k;
            // (no split records in this form; the record index is opaque so that both forms compile the same
            // solve_one — fp32 contraction / packing decisions otherwise differ between them)
            long long rec = -1;
            asm volatile("" : "+s"(rec));
            if (!Pv.active || Pv.active[b]) solve_one<N, KSM, R, true, false, RS>(P, G, wsb, wv, b, rec);   // rollout: skip finished
        }
        queue_exit(q);
    }
}

#include "lane_solve.inc"

// ------------------------------------------------------------------------------------------------
// eval kernel ("Jacobian sweep"): f, grad f, c, J, cl, cu, goal_eff, row_active at given u.
//   One instance per 16-lane group (4 instances per wave, 16 per 256-thread workgroup): the per-instance
//   set-up (select_obs ballots, detour, the rollout V = E x0 + G u, the N sin/cos/atan2 of the state pass)
//   runs on a few lanes of each group at once, so its instruction stream is shared by 4 instances instead
//   of being paid per wave; lane t of a group owns rows t, t + 16, ... and J columns t (+ 16), and a J row
//   store is 4 contiguous 15-double runs (the rows of one instance are adjacent, so an instance's J block is
//   written front to back).
// ------------------------------------------------------------------------------------------------
constexpr int GLANES = 16;                          // lanes per instance (one DPP row)
constexpr int GROUPS_PER_BLOCK = WAVE * WAVES_PER_BLOCK / GLANES;

// per-group eval workspace (doubles)
template <int N>
struct GWS {
    double* rcoef;  // mr4 x 4
    uint8_t* rgen;  // mr4 x 4
    double* V;      // NG
    double* gfg;    // NG   d f / d V
    double* CT;     // N+1
    double* ST;     // N+1
    double* uv;     // nu   the instance's u
    double* obs;    // circles 3*nc_max, ellipses 5*ne_max, then qa, qb, qc, ek (4*ne_max)
};
// the group stride is 4 (mod 16) doubles: the 4 groups of a wave read their rcoef rows (32-byte broadcasts)
// from disjoint LDS banks
template <int N>
__host__ __device__ constexpr int gws_doubles(int nc_max, int ne_max, int mr4)
{
    const int d = 4 * mr4 + mr4 / 2 + 2 * Dim<N>::NG + 2 * (N + 1) + Dim<N>::nu + 3 * nc_max + 9 * ne_max;
    return d + ((4 - d) % 16 + 16) % 16;
}
template <int N>
__device__ GWS<N> carve_g(double* p, int nc_max, int ne_max, int mr4)
{
    GWS<N> w;
    w.rcoef = p; p += 4 * mr4;   // 32-byte rows
    w.rgen = reinterpret_cast<uint8_t*>(p); p += mr4 / 2;   // mr4 is a multiple of 4: 16-byte row quads
    w.V = p; p += Dim<N>::NG;
    w.gfg = p; p += Dim<N>::NG;
    w.CT = p; p += N + 1;
    w.ST = p; p += N + 1;
    w.uv = p; p += Dim<N>::nu;
    w.obs = p;
    return w;
}

// global-memory views of output pointers (plain pointers read from the LDS copy of KP would be flat
// accesses, whose stores also hold the LDS counter that every following LDS wait drains)
typedef __attribute__((address_space(1))) double gdouble;
typedef __attribute__((address_space(1))) int8_t gint8;
__device__ __forceinline__ gdouble* gptr(double* p) { return (gdouble*)p; }
__device__ __forceinline__ gint8* gptr(int8_t* p) { return (gint8*)p; }
__device__ __forceinline__ const gdouble* gptr(const double* p) { return (const gdouble*)p; }

// the 16 ballot bits of this lane's group
__device__ __forceinline__ unsigned gballot(bool x)
{
    return (unsigned)(__ballot(x) >> (threadIdx.x & (WAVE - GLANES))) & 0xFFFFu;
}
// sum over the 16 lanes of a DPP row (every lane receives it)
__device__ __forceinline__ double gsum16(double v)
{
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    v += dpp<0x141>(v);
    v += dpp<0x140>(v);
    return v;
}

// one row family of the eval layout for a group: item i = (step k, slot) with cnt slots per step at row offset
// loff within the step; CIR / ELP slots at or past nsel (selected obstacles) are inactive rows
template <int N, int TYPE>
__device__ __forceinline__ void eval_rows(const KP& P, const GWS<N>& w, long long b, int t, int legv, int nsel, int cnt,
                                          int loff)
{
    const size_t mm = (size_t)P.m_max;
    const int total = N * cnt;
    for (int i = t; i < total; i += GLANES) {
        const int k = cnt == 1 ? i : i / cnt, slot = i - k * cnt;
        const int r = k * P.rps + loff + slot;
        const bool act = (TYPE != R_CIR && TYPE != R_ELP) || slot < nsel;
        RowInfo ri;
        ri.type = TYPE;
        ri.k = k;
        ri.slot = slot;
        double cf[4];
        int gn[4];
        double c = row_eval<N, true>(P, ri, w.V, w.CT, w.ST, w.obs, 0.0, cf, gn);
        if (!act) {
            c = 0.0;
            cf[0] = cf[1] = cf[2] = cf[3] = 0.0;
            gn[0] = gn[1] = gn[2] = gn[3] = 0;
            ri.type = R_NONE;
        }
        st4(w.rcoef + 4 * r, cf[0], cf[1], cf[2], cf[3]);
        *reinterpret_cast<uint32_t*>(w.rgen + 4 * r) =
            (uint32_t)gn[0] | ((uint32_t)gn[1] << 8) | ((uint32_t)gn[2] << 16) | ((uint32_t)gn[3] << 24);
        double clv, cuv;
        row_bounds(P, ri, legv, clv, cuv);
        if (P.c_out) gptr(P.c_out)[b * mm + r] = c;
        if (P.cl_out) gptr(P.cl_out)[b * mm + r] = clv;
        if (P.cu_out) gptr(P.cu_out)[b * mm + r] = cuv;
        if (P.active_out) gptr(P.active_out)[b * mm + r] = act;
    }
}

template <int N>
__device__ __forceinline__ void eval_group_one(const KP& P, const GWS<N>& w, const double* G, const double* E, long long b,
                                               int t)
{
    using D = Dim<N>;
    constexpr int nu = D::nu, NTU = D::NTU, NCP = D::NCPU, NG = D::NG;
    const gdouble* x0 = gptr(P.x0) + 5 * b;
    const int legv = P.leg[b];
    const int ncr = P.nc[b];
    const int ner = P.ne ? P.ne[b] : 0;
    const double x0v0 = x0[0], x0v1 = x0[1];
    const double g0 = gptr(P.goal)[2 * b], g1 = gptr(P.goal)[2 * b + 1];
    // select_obs (MPC_LIP_modi.py:325-338): keep order, compact into the first slots (16 slots per pass)
    int ncs = 0, nes = 0;
    for (int base = 0; base < P.nc_max; base += GLANES) {
        const int j = base + t;
        const bool valid = j < ncr && j < P.nc_max;
        double c0 = 0, c1 = 0, c2 = 0;
        if (valid) {
            const gdouble* c = gptr(P.cir) + ((size_t)b * P.nc_max + j) * 3;
            c0 = c[0]; c1 = c[1]; c2 = c[2];
        }
        const double d = (x0v0 - c0) * (x0v0 - c0) + (x0v1 - c1) * (x0v1 - c1) - c2 * c2;
        const bool keep = valid && (!P.select_obs || d <= P.detect_r2);
        const unsigned m = gballot(keep);
        const int pos = ncs + __builtin_popcount(m & ((1u << t) - 1u));
        if (keep) {
            w.obs[3 * pos + 0] = c0;
            w.obs[3 * pos + 1] = c1;
            w.obs[3 * pos + 2] = c2;
        }
        ncs += __builtin_popcount(m);
    }
    for (int base = 0; base < P.ne_max; base += GLANES) {
        const int j = base + t;
        const bool valid = j < ner && j < P.ne_max;
        double e[5] = {0, 0, 0, 0, 0};
        if (valid) {
            const gdouble* ep = gptr(P.elp) + ((size_t)b * P.ne_max + j) * 5;
            for (int i = 0; i < 5; ++i) e[i] = ep[i];
        }
        const double rmax = e[2] > e[3] ? e[2] : e[3];
        const double d = (x0v0 - e[0]) * (x0v0 - e[0]) + (x0v1 - e[1]) * (x0v1 - e[1]) - rmax * rmax;
        const bool keep = valid && (!P.select_obs || d <= P.detect_r2);
        const unsigned m = gballot(keep);
        const int pos = nes + __builtin_popcount(m & ((1u << t) - 1u));
        if (keep) {
            double* o = w.obs + 3 * P.nc_max + 5 * pos;
            for (int i = 0; i < 5; ++i) o[i] = e[i];
            double ce, se;
            sincos(e[4], &se, &ce);
            double* qq = w.obs + 3 * P.nc_max + 5 * P.ne_max;
            qq[pos] = (e[3] * ce) * (e[3] * ce) + (e[2] * se) * (e[2] * se);
            qq[P.ne_max + pos] = 2 * ce * se * (e[3] * e[3] - e[2] * e[2]);
            qq[2 * P.ne_max + pos] = (e[3] * se) * (e[3] * se) + (e[2] * ce) * (e[2] * ce);
            qq[3 * P.ne_max + pos] = (e[3] * e[2]) * (e[3] * e[2]);
        }
        nes += __builtin_popcount(m);
    }
    // the instance's u (the rollout below reads it from LDS)
    for (int j = t; j < nu; j += GLANES) w.uv[j] = gptr(P.u0)[(size_t)b * nu + j];
    wave_sync();
    // detour goal (MPC_LIP_modi.py:247-271): first selected circle that triggers
    double gxg = g0, gyg = g1;
    bool found = false;
    for (int base = 0; P.detour && !found && base < ncs; base += GLANES) {
        const int j = base + t;
        bool fire = false;
        double nx = 0, ny = 0;
        if (j < ncs) {
            const double* c = w.obs + 3 * j;
            const double cen = fma(x0v0 - c[0], x0v0 - c[0], (x0v1 - c[1]) * (x0v1 - c[1]));
            const double gd = fma(x0v0 - g0, x0v0 - g0, (x0v1 - g1) * (x0v1 - g1));
            if (cen < gd && cen < 9 * c[2] * c[2]) {
                const double th = latan2(g1 - x0v1, g0 - x0v0);
                const double al = latan2(c[1] - x0v1, c[0] - x0v0);
                double dd = th - al;
                if (dd < 0 && fabs(dd) > M_PI)
                    dd += 2 * M_PI;
                else if (dd > 0 && fabs(dd) > M_PI)
                    dd -= 2 * M_PI;
                if (fabs(dd) < M_PI / 12) {
                    fire = true;
                    const double na = dd < 0 ? th - M_PI / 12 : th + M_PI / 12;
                    const double rr = sqrt(gd);
                    double sn, cs;
                    lsincos(na, &sn, &cs);
                    nx = fma(rr, cs, x0v0);   // (explicit fma: every kernel's detour goal rounds alike)
                    ny = fma(rr, sn, x0v1);
                }
            }
        }
        const unsigned m = gballot(fire);
        if (m) {
            const int first = __builtin_ctz(m);
            gxg = __shfl(nx, first, GLANES);
            gyg = __shfl(ny, first, GLANES);
            found = true;
        }
    }
    // V = E x0 + G u (the reference's rollout of u)
    double xb[5];
#pragma unroll
    for (int c = 0; c < 5; ++c) xb[c] = x0[c];
    for (int g = t; g < NG; g += GLANES) {
        double v = 0.0;
#pragma unroll
        for (int c = 0; c < 5; ++c) v += E[g * 5 + c] * xb[c];
        const double* gr = G + g * NCP;
#pragma unroll
        for (int j = 0; j < nu; ++j) v += gr[j] * w.uv[j];
        w.V[g] = v;
        w.gfg[g] = 0.0;
    }
    wave_sync();
    // state pass: lanes 1..N own x_k (cos/sin of theta_k, the objective term f_k and its gradient)
    double fk = 0.0;
    if (t >= 1 && t <= N) {
        const int k = t;
        const double th = w.V[gx(k, 4)];
        double s_, c_;
        lsincos(th, &s_, &c_);
        w.CT[k] = c_;
        w.ST[k] = s_;
        const double px = w.V[gx(k, 0)], py = w.V[gx(k, 1)];
        const double wk = P.q + (k == 1 ? P.p : 0.0);
        const double ex = px - gxg, ey = py - gyg;
        const double dxg = gxg - px, dyg = gyg - py;
        const double phi = th - latan2(dyg, dxg);
        fk = wk * (ex * ex + ey * ey) + P.r * phi * phi;
        const double rho2 = dxg * dxg + dyg * dyg;
        // (p = goal exactly: the target heading's derivatives are 0)
        // (explicit fma: the sweep kernel's copy of these sums must contract the same way)
        const double q0 = rho2 > 0.0 ? -dyg / rho2 : 0.0, q1 = rho2 > 0.0 ? dxg / rho2 : 0.0;
        w.gfg[gx(k, 0)] = fma(2 * P.r * phi, q0, 2 * wk * ex);
        w.gfg[gx(k, 1)] = fma(2 * P.r * phi, q1, 2 * wk * ey);
        w.gfg[gx(k, 4)] = 2 * P.r * phi;
    }
    const double f = gsum16(fk);
    wave_sync();
    // rows: values, bounds, activity, generator-form Jacobian rows — one pass per row family (the family is a
    // compile-time constant in each pass, so no per-row decode and no divergent switch over the families)
    const size_t mm = (size_t)P.m_max;
    {
        const int nc = P.nc_max, ne = P.ne_max, lo = 2 + nc + ne;
        eval_rows<N, R_VBX>(P, w, b, t, legv, 0, 1, 0);
        eval_rows<N, R_VBY>(P, w, b, t, legv, 0, 1, 1);
        if (nc) eval_rows<N, R_CIR>(P, w, b, t, legv, ncs, nc, 2);
        if (ne) eval_rows<N, R_ELP>(P, w, b, t, legv, nes, ne, 2 + nc);
        eval_rows<N, R_LEG>(P, w, b, t, legv, 0, 1, lo);
        eval_rows<N, R_DTH>(P, w, b, t, legv, 0, 1, lo + 1);
        if (P.rps > lo + 2) eval_rows<N, R_FEN>(P, w, b, t, legv, 0, 1, lo + 2);
        for (int r = P.m_max + t; r < P.mr4; r += GLANES) {   // padding rows: zero coefficients for the J steps
            st4(w.rcoef + 4 * r, 0.0, 0.0, 0.0, 0.0);
            *reinterpret_cast<uint32_t*>(w.rgen + 4 * r) = 0u;
        }
    }
    wave_sync();
    // J rows (dense, u-space): lane t writes columns t (+ 16)
    if (P.J_out) {
        gdouble* Jb = gptr(P.J_out + (size_t)b * mm * nu);
        // 4 rows per step (mr4 is a multiple of 4): every LDS read of the step is issued before the FMAs
        for (int r0 = 0; r0 < P.m_max; r0 += 4) {
            const uint4 pk4 = *reinterpret_cast<const uint4*>(w.rgen + 4 * r0);
            const uint32_t pk[4] = {pk4.x, pk4.y, pk4.z, pk4.w};
            double cf[4][4];
#pragma unroll
            for (int i = 0; i < 4; ++i) ld4(w.rcoef + 4 * (r0 + i), cf[i][0], cf[i][1], cf[i][2], cf[i][3]);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = r0 + i;
#pragma unroll
                for (int T = 0; T < NTU; ++T) {
                    const int j = GLANES * T + t;
                    const double v = cf[i][0] * G[gen_i(pk[i], 0) * NCP + j] + cf[i][1] * G[gen_i(pk[i], 1) * NCP + j] +
                                     cf[i][2] * G[gen_i(pk[i], 2) * NCP + j] + cf[i][3] * G[gen_i(pk[i], 3) * NCP + j];
                    if (j < nu && r < P.m_max) Jb[(size_t)r * nu + j] = v;
                }
            }
        }
    }
    // grad f = G^T (d f / d V) (x_0 and the p_k generators carry no objective gradient)
    if (P.grad_out) {
#pragma unroll
        for (int T = 0; T < NTU; ++T) {
            const int j = GLANES * T + t;
            double gf = 0.0;
            for (int g = 8; g < NG; ++g) gf += G[g * NCP + j] * w.gfg[g];
            if (j < nu) gptr(P.grad_out)[b * nu + j] = gf;
        }
    }
    if (t == 0) {
        if (P.f_out) gptr(P.f_out)[b] = f;
        if (P.goal_eff_out) {
            gptr(P.goal_eff_out)[2 * b] = gxg;
            gptr(P.goal_eff_out)[2 * b + 1] = gyg;
        }
    }
    wave_sync();
}

template <int N>
__global__ __launch_bounds__(256) void eval_kernel(KP Pv)
{
    using D = Dim<N>;
    constexpr int NCP = D::NCPU;
    constexpr int NG = D::NG;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    // kernel parameters live in LDS: keeps ~90 kernarg SGPRs from being pinned across the sweep
    KP* Ps = reinterpret_cast<KP*>(smem);
    double* G = smem + KP_DOUBLES;
    double* E = G + NG * NCP;
    double* wsb = E + NG * 5 + ((NG * 5) & 1);
    if (threadIdx.x == 0) *Ps = Pv;
    for (int i = threadIdx.x; i < NG * NCP; i += blockDim.x) G[i] = Pv.G[i];
    for (int i = threadIdx.x; i < NG * 5; i += blockDim.x) E[i] = Pv.E[i];
    __syncthreads();
    const KP& P = *Ps;
    const int gi = threadIdx.x / GLANES, t = threadIdx.x & (GLANES - 1);
    const GWS<N> w = carve_g<N>(wsb + (size_t)gi * gws_doubles<N>(P.nc_max, P.ne_max, P.mr4), P.nc_max, P.ne_max, P.mr4);
    // grid-stride over instances (the G/E staging above is paid once per workgroup); the 4 groups of a wave
    // take 4 consecutive instances
    for (long long b0 = (long long)blockIdx.x * GROUPS_PER_BLOCK; b0 < P.B; b0 += (long long)gridDim.x * GROUPS_PER_BLOCK) {
        const long long b = b0 + gi;
        if (b < P.B) eval_group_one<N>(P, w, G, E, b, t);
    }
}

// ------------------------------------------------------------------------------------------------
// sweep kernel: the eval hook at N = 3 with circle slots only (cfg2's shape, the bench's Jacobian sweep).
//   The dense J block (m x 5N doubles) is ~90 % of the bytes an evaluation writes, so the kernel is built
//   around writing it with full-width stores, with the per-instance set-up shared by 64 instances per
//   instruction stream:
//   Phase A (lane = instance, 64 per wave): inputs, select_obs (in-order compaction by rank selects), detour,
//     the rollout V = E x0 + G u over the structurally non-zero terms of G (x_k depends on u_0..u_{k-1}, p_k on
//     u_0..u_k; the skipped products are exact zeros), the state pass, f, grad f, and per row the value,
//     bounds and activity (per-lane stores) and the generator-form coefficients (to LDS).
//   Phase B (wave-cooperative): element e = lane + 64 s of an instance's J block (row e / 5N, column e % 5N)
//     is sum_i cf[row][i] * G[gen_i(row)][col]; the G values depend on e only, so one element step runs over
//     all the blocks with 4 G values in registers, and one store instruction writes 512 contiguous bytes.
//   A chunk is CH = 32 instances per wave (lanes 32..63 repeat lanes 0..31 and store nothing), two waves per
//   workgroup sharing one G/E copy: 2048 waves at B = 65,536, two per SIMD, so one wave's set-up runs under the
//   other's J stores (the LDS of a 64-instance chunk had allowed one wave per SIMD).  The coefficient LDS holds
//   CH / 2 instances: the two halves of a chunk take turns.  The sums are eval_kernel's, term for term and in
//   the same order (the outputs are bit-identical, tests/test_gpu.py).
// ------------------------------------------------------------------------------------------------
#ifndef SWEEP_SHAPE_DEFAULT
#define SWEEP_SHAPE_DEFAULT 322
#endif
template <int NC, bool FEN>
struct SweepL {
    static constexpr int N = 3, nu = 15, NG = 32, NCPU = 16;
    static constexpr int rps = 4 + NC + (FEN ? 1 : 0);
    static constexpr int m = N * rps;
    static constexpr int mn = m * nu;
    static constexpr int S = (mn + WAVE - 1) / WAVE;   // J element steps per instance
    // one instance slot of the coefficient LDS in dwords: >= 8m and = 52 (mod 64), so the 16 lanes of a
    // b128 store pass write disjoint bank quads
    static constexpr int SLOTW = 8 * m + (((52 - 8 * m) % 64) + 64) % 64;
    static constexpr int SLOTD = SLOTW / 2;
    static constexpr int GL = NG * NCPU + NG * 5;      // LDS copy of G and E (672 doubles: slots stay aligned)
};
typedef __attribute__((address_space(3))) double ldouble;

// generator rows of row rr of step k in the eval layout [vbx, vby, circles, leg, dtheta, (f_en)] (-1: none)
template <int NC, bool FEN>
__device__ __forceinline__ void sweep_gens(int rr, int k, int (&g)[4])
{
    g[0] = g[1] = g[2] = g[3] = -1;
    if (rr < 2 || (FEN && rr == 4 + NC)) {
        g[0] = gx(k + 1, 2); g[1] = gx(k + 1, 3); g[2] = gx(k + 1, 4);
        if (rr >= 2) g[3] = gp(k, 2);
    } else if (rr < 2 + NC) {
        g[0] = gx(k + 1, 0); g[1] = gx(k + 1, 1); g[2] = gx(k, 0); g[3] = gx(k, 1);
    } else if (rr == 2 + NC) {
        g[0] = gx(k, 0); g[1] = gx(k, 1); g[2] = gp(k, 0); g[3] = gp(k, 1);
    } else {
        g[0] = gp(k, 2);
    }
}

template <int NC, bool FEN, int CH, int WPG>
__global__ __launch_bounds__(WAVE * WPG, 2) void sweep_kernel(KP Pv)
{
    using L = SweepL<NC, FEN>;
    constexpr int N = L::N, nu = L::nu, NG = L::NG, NCPU = L::NCPU, m = L::m, rps = L::rps, S = L::S;
    constexpr int mn = L::mn, SLOTD = L::SLOTD;
    constexpr int QI = CH / 2;   // instances per coefficient pass (two passes per chunk)
    constexpr int NO = NC > 0 ? 3 * NC : 1;
    static_assert(CH == 64 || CH == 32, "instances per wave");
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* Gl = smem;
    const int wv = threadIdx.x / WAVE, lane = threadIdx.x % WAVE;
    double* cfs = smem + L::GL + (size_t)wv * QI * SLOTD;
    for (int i = threadIdx.x; i < NG * NCPU; i += WAVE * WPG) Gl[i] = Pv.G[i];
    for (int i = threadIdx.x; i < NG * 5; i += WAVE * WPG) Gl[NG * NCPU + i] = Pv.E[i];
    __syncthreads();
    const double* const El = Gl + NG * NCPU;
    gdouble* const Jo = Pv.J_out ? gptr(Pv.J_out) : nullptr;
    for (long long b0 = ((long long)blockIdx.x * WPG + wv) * CH; b0 < Pv.B; b0 += (long long)gridDim.x * WPG * CH) {
        // the parameters are read from the kernarg segment where they are used (a laundered constant-space
        // pointer per chunk): ~100 kernarg SGPRs otherwise stay live across the chunk and spill
        const __attribute__((address_space(4))) char* kq =
            (const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(kq));
        const KP& P = *(const KP*)(const __attribute__((address_space(4))) KP*)kq;
        // ---------------- phase A: this lane's instance
        // lane % CH owns an instance; lanes >= CH repeat it (same values, no stores): the wave keeps 64 lanes
        // while a chunk is CH instances, so a batch makes B / CH waves (latency of one chunk's set-up hidden
        // behind another's J stores)
        const long long b = b0 + lane % CH;
        const bool live = lane < CH && b < P.B;
        const long long bl = b < P.B ? b : P.B - 1;
        double x0v[5], u[nu];
        const gdouble* x0p = gptr(P.x0) + 5 * bl;
#pragma unroll
        for (int c = 0; c < 5; ++c) x0v[c] = x0p[c];
        const gdouble* up = gptr(P.u0) + (size_t)nu * bl;
#pragma unroll
        for (int j = 0; j < nu; ++j) u[j] = up[j];
        const double g0 = gptr(P.goal)[2 * bl], g1 = gptr(P.goal)[2 * bl + 1];
        const int legv = P.leg[bl];
        const int ncr = P.nc[bl];
        // select_obs (MPC_LIP_modi.py:325-338): the kept circles in input order, compacted by rank
        double obs[NO];
#pragma unroll
        for (int i = 0; i < NO; ++i) obs[i] = 0.0;
        int nsel = 0;
#pragma unroll
        for (int jc = 0; jc < NC; ++jc) {
            const bool valid = jc < ncr;
            double c0 = 0, c1 = 0, c2 = 0;
            if (valid) {
                const gdouble* c = gptr(P.cir) + ((size_t)bl * NC + jc) * 3;
                c0 = c[0]; c1 = c[1]; c2 = c[2];
            }
            const double d = (x0v[0] - c0) * (x0v[0] - c0) + (x0v[1] - c1) * (x0v[1] - c1) - c2 * c2;
            const bool keep = valid && (!P.select_obs || d <= P.detect_r2);
#pragma unroll
            for (int sl = 0; sl <= jc; ++sl) {
                const bool here = keep && nsel == sl;
                obs[3 * sl + 0] = here ? c0 : obs[3 * sl + 0];
                obs[3 * sl + 1] = here ? c1 : obs[3 * sl + 1];
                obs[3 * sl + 2] = here ? c2 : obs[3 * sl + 2];
            }
            nsel += keep ? 1 : 0;
        }
        // detour goal (MPC_LIP_modi.py:247-271): the first selected circle that triggers.  Branch-free: the heading
        // to the goal and every circle's bearing are independent (one instruction stream, interleaved), then the
        // first firing circle's side picks the new heading (same functions, same values as eval_kernel)
        double gxg = g0, gyg = g1;
        if (P.detour) {
            const double gd = fma(x0v[0] - g0, x0v[0] - g0, (x0v[1] - g1) * (x0v[1] - g1));
            const double th = latan2(g1 - x0v[1], g0 - x0v[0]);
            bool found = false;
            double na = 0.0;
#pragma unroll
            for (int sl = 0; sl < NC; ++sl) {
                const double* c = obs + 3 * sl;
                const double cen = fma(x0v[0] - c[0], x0v[0] - c[0], (x0v[1] - c[1]) * (x0v[1] - c[1]));
                const double al = latan2(c[1] - x0v[1], c[0] - x0v[0]);
                double dd = th - al;
                if (dd < 0 && fabs(dd) > M_PI)
                    dd += 2 * M_PI;
                else if (dd > 0 && fabs(dd) > M_PI)
                    dd -= 2 * M_PI;
                const bool fire = sl < nsel && cen < gd && cen < 9 * c[2] * c[2] && fabs(dd) < M_PI / 12;
                na = (fire && !found) ? (dd < 0 ? th - M_PI / 12 : th + M_PI / 12) : na;
                found = found || fire;
            }
            if (found) {
                const double rr = sqrt(gd);
                double sn, cs;
                lsincos(na, &sn, &cs);
                gxg = fma(rr, cs, x0v[0]);
                gyg = fma(rr, sn, x0v[1]);
            }
        }
        // V = E x0 + G u over the structural non-zeros of G (x_k: u_0..u_{k-1}; p_k: u_0..u_k)
        double V[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const int k = g / 8, c = g % 8;
            const int lim = c < 5 ? 5 * k : (k < N ? 5 * (k + 1) : 0);
            if (c >= 5 && k == N) {   // p_N: not a generator of any row
                V[g] = 0.0;
                continue;
            }
            // one generator row at a time: its (broadcast) LDS reads, then its FMAs — the laundered offset keeps the
            // reads from being hoisted into one block of hundreds of live VGPRs
            int og = g * NCPU, oe = g * 5;
            asm volatile("" : "+v"(og), "+v"(oe));
            const ldouble* gr = (const ldouble*)Gl + og;
            const ldouble* er = (const ldouble*)El + oe;
            double v = 0.0;
#pragma unroll
            for (int cc = 0; cc < 5; ++cc) v += er[cc] * x0v[cc];
#pragma unroll
            for (int j = 0; j < lim; ++j) v += gr[j] * u[j];
            asm volatile("" : "+v"(v));   // computed here (not sunk to its uses, which would keep the reads live)
            V[g] = v;
        }
        // state pass: cos/sin theta_k, the objective terms f_k and d f / d V
        double CT[N + 1], ST[N + 1], fk[N + 1], gfg[N + 1][3];
        CT[0] = ST[0] = fk[0] = 0.0;
#pragma unroll
        for (int k = 1; k <= N; ++k) {
            const double th = V[gx(k, 4)];
            double s_, c_;
            lsincos(th, &s_, &c_);
            CT[k] = c_;
            ST[k] = s_;
            const double px = V[gx(k, 0)], py = V[gx(k, 1)];
            const double wk = P.q + (k == 1 ? P.p : 0.0);
            const double ex = px - gxg, ey = py - gyg;
            const double dxg = gxg - px, dyg = gyg - py;
            const double phi = th - latan2(dyg, dxg);
            fk[k] = wk * (ex * ex + ey * ey) + P.r * phi * phi;
            const double rho2 = dxg * dxg + dyg * dyg;
            const double q0 = rho2 > 0.0 ? -dyg / rho2 : 0.0, q1 = rho2 > 0.0 ? dxg / rho2 : 0.0;
            gfg[k][0] = fma(2 * P.r * phi, q0, 2 * wk * ex);   // (eval_group_one's sums, contracted alike)
            gfg[k][1] = fma(2 * P.r * phi, q1, 2 * wk * ey);
            gfg[k][2] = 2 * P.r * phi;
        }
        if (live) {
            // eval_kernel's 16-lane butterfly sum of f_1..f_3 is f_1 + (f_2 + f_3)
            if (P.f_out) gptr(P.f_out)[b] = fk[1] + (fk[2] + fk[3]);
            if (P.goal_eff_out) {
                gptr(P.goal_eff_out)[2 * b] = gxg;
                gptr(P.goal_eff_out)[2 * b + 1] = gyg;
            }
            // grad f = G^T (d f / d V): the non-zero terms of eval_kernel's sum over g = 8..NG-1, in its order
            if (P.grad_out) {
#pragma unroll 1
                for (int j = 0; j < nu; ++j) {   // a loop: 9 broadcast reads per column, not 135 at once
                    const ldouble* gc = (const ldouble*)Gl + j;
                    double gf = 0.0;
#pragma unroll
                    for (int k = 1; k <= N; ++k) {
                        gf += gc[gx(k, 0) * NCPU] * gfg[k][0];
                        gf += gc[gx(k, 1) * NCPU] * gfg[k][1];
                        gf += gc[gx(k, 4) * NCPU] * gfg[k][2];
                    }
                    gptr(P.grad_out)[(size_t)b * nu + j] = gf;
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        // rows: the lanes of one half at a time write their coefficients, then the wave writes those 32 J blocks
#pragma unroll 1
        for (int h = 0; h < 2; ++h) {
            // the row arithmetic of each half stays in its pass (hoisted out of this loop it is live across
            // phase B and spills)
#pragma unroll
            for (int g = 0; g < NG; ++g) asm volatile("" : "+v"(V[g]));
#pragma unroll
            for (int k = 0; k <= N; ++k) asm volatile("" : "+v"(CT[k]), "+v"(ST[k]));
#pragma unroll
            for (int i = 0; i < NO; ++i) asm volatile("" : "+v"(obs[i]));
            if (lane < CH && lane / QI == h) {
                double* slot = cfs + (size_t)(lane % QI) * SLOTD;
#pragma unroll
                for (int k = 0; k < N; ++k) {
#pragma unroll
                    for (int rr = 0; rr < rps; ++rr) {
                        const int r = k * rps + rr;
                        RowInfo ri;
                        ri.k = k;
                        ri.slot = rr >= 2 && rr < 2 + NC ? rr - 2 : 0;
                        ri.type = rr == 0 ? R_VBX
                                : rr == 1 ? R_VBY
                                : rr < 2 + NC ? R_CIR
                                : rr == 2 + NC ? R_LEG
                                : rr == 3 + NC ? R_DTH : R_FEN;
                        const bool act = ri.type != R_CIR || ri.slot < nsel;
                        double cf[4];
                        int gn[4];
                        double c = row_eval<N, true>(P, ri, V, CT, ST, obs, 0.0, cf, gn);
                        if (!act) {
                            c = 0.0;
                            cf[0] = cf[1] = cf[2] = cf[3] = 0.0;
                            ri.type = R_NONE;
                        }
                        if (live) {
                            const size_t o = (size_t)b * m + r;
                            if (P.c_out) gptr(P.c_out)[o] = c;
                            if (P.cl_out || P.cu_out) {
                                double clv, cuv;
                                row_bounds(P, ri, legv, clv, cuv);
                                if (P.cl_out) gptr(P.cl_out)[o] = clv;
                                if (P.cu_out) gptr(P.cu_out)[o] = cuv;
                            }
                            if (P.active_out) gptr(P.active_out)[o] = act;
                        }
                        if (Jo) st4(slot + 4 * r, cf[0], cf[1], cf[2], cf[3]);
                    }
                }
            }
            if (!Jo) continue;
            wave_sync();
            // ---------------- phase B: the J blocks of this half's instances, one element step s at a time (lane
            // element e = lane + 64 s: row r = e / 5N, column j = e % 5N, the same in every block), 8 blocks per pass
            const long long bh = b0 + h * QI;
            const int cnt = P.B - bh < QI ? (int)(P.B - bh) : QI;
#pragma unroll 1
            for (int s = 0; s < S; ++s) {
                const int e = lane + WAVE * s;
                if (e < mn) {
                    const int r = e / nu, j = e - r * nu;
                    int g[4];
                    sweep_gens<NC, FEN>(r % rps, r / rps, g);
                    double gv[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) gv[q] = g[q] >= 0 ? Gl[g[q] * NCPU + j] : 0.0;
                    const double* cfr = cfs + 4 * r;
                    gdouble* Jp = Jo + (size_t)bh * mn + e;
                    int i = 0;
                    for (; i + 8 <= cnt; i += 8) {
                        double a[8][4];
#pragma unroll
                        for (int q = 0; q < 8; ++q) ld4(cfr + (size_t)(i + q) * SLOTD, a[q][0], a[q][1], a[q][2], a[q][3]);
#pragma unroll
                        for (int q = 0; q < 8; ++q)
                            Jp[(size_t)(i + q) * mn] = a[q][0] * gv[0] + a[q][1] * gv[1] + a[q][2] * gv[2] + a[q][3] * gv[3];
                    }
                    for (; i < cnt; ++i) {
                        double a0, a1, a2, a3;
                        ld4(cfr + (size_t)i * SLOTD, a0, a1, a2, a3);
                        Jp[(size_t)i * mn] = a0 * gv[0] + a1 * gv[1] + a2 * gv[2] + a3 * gv[3];
                    }
                }
            }
            wave_sync();
        }
    }
}


// ================================================================================================
// DD variant: unicycle MPC-CBF (MPC_DD_sig_step.py:123-193 set-up, 320-572 LIP_Prob)
//   x = [px, py, th], u = [v_0, w_0, ..., v_{N-1}, w_{N-1}] (n = 2N),
//   x_{i+1} = x_i + [T v_i cos th_i, T v_i sin th_i, w_i].
// The dynamics are not affine in u, so there is no generator space: each evaluation rolls the N steps
// out (state lanes, one sincos per lane + readlane prefix sums), every row lane writes its full
// Jacobian row (n <= 12, closed forms of cal_dx_du :534-566) to LDS, and the exact Hessian adds the
// rollout's second derivatives.  The interior-point logic (barrier, filter, inertia correction) is the
// same as solve_kernel's.
// Solve rows per step: [cbf circle slots, cbf ellipse slots, v + s w <= v_max, v - s w <= v_max,
// v in [v_min, v_max], w in [-w_max, w_max]] (f_en split and the reference's variable bounds as rows),
// then N objective pseudo-rows.  Eval rows per step: the reference's [cbf..., f_en = s|w| + v].
// ================================================================================================
enum DDType { D_CIR = 0, D_ELP, D_FENP, D_FENM, D_VB, D_WB, D_NONE, D_OBJ, D_FEN };
enum { DK_GM1 = 0, DK_S, DK_Q, DK_P, DK_R, DK_GX, DK_GY, DK_T, DK_TT, DK_LU0, DK_LU1, DK_THMAX, DK_THMIN,
       DK_MACT, DK_NBL, DK_TOL, DK_ACCTOL, DK_X0, DK_X1, DK_X2, DK_COUNT };
constexpr int DD_ST = 8;   // per-step stride of the state table: px, py, th, T cos th, T sin th

template <int N>
struct DDW {
    double* cst;   // DK_COUNT (rounded to 24)
    double* STa;   // (N+1) x DD_ST  state tables (current / trial swap roles)
    double* STb;
    double* Ua;    // 16 decision (current / trial)
    double* Ub;
    double* dU;    // 16 step
    double* Jd;    // mo4 x 16 Jacobian rows
    double* ry;    // mo4
    double* rsig;  // mo4
    double* rw;    // mo4
    double* hl;    // (N+1) x 8: Hessian parts per step [h00 h01 h11 h02 h12 h22 g0 g1]
    double* hobj;  // (N+1) x 8: objective contributions (written by the OBJ rows)
    double* obs6;  // (nobs + 1) x 6
    double* K;     // 16 x 17
    double* rclo;  // mo4
    double* rcuo;  // mo4
};

template <int N>
__host__ __device__ constexpr int ddw_doubles(int nobs, int mo4)
{
    int d = 24 + 2 * (N + 1) * DD_ST + 3 * 16 + 16 * mo4 + 3 * mo4 + 2 * 8 * (N + 1) + 6 * (nobs + 1) + 16 * 17 +
            2 * mo4;
    return (d + 3) & ~3;
}

template <int N>
__device__ DDW<N> carve_dd(double* p, int nobs, int mo4)
{
    DDW<N> w;
    w.Jd = p; p += 16 * mo4;   // first: 32-byte aligned
    w.cst = p; p += 24;
    w.STa = p; p += (N + 1) * DD_ST;
    w.STb = p; p += (N + 1) * DD_ST;
    w.Ua = p; p += 16;
    w.Ub = p; p += 16;
    w.dU = p; p += 16;
    w.ry = p; p += mo4;
    w.rsig = p; p += mo4;
    w.rw = p; p += mo4;
    w.hl = p; p += 8 * (N + 1);
    w.hobj = p; p += 8 * (N + 1);
    w.obs6 = p; p += 6 * (nobs + 1);
    w.K = p; p += 16 * 17;
    w.rclo = p; p += mo4;
    w.rcuo = p;
    return w;
}

// row decode (solve layout split = true: rps = nobs + 4; eval layout: rps = nobs + 1)
__device__ __forceinline__ void dd_decode(int r, int rps, int m, int nc_max, int ne_max, int nc, int ne, bool split,
                                          int& type, int& k, int& oi)
{
    type = D_NONE;
    k = 0;
    oi = 0;
    if (r >= m) return;
    k = r / rps;
    const int l = r - k * rps;
    const int nobs = nc_max + ne_max;
    if (l < nc_max) {
        type = l < nc ? D_CIR : D_NONE;
        oi = l;
    } else if (l < nobs) {
        type = (l - nc_max) < ne ? D_ELP : D_NONE;
        oi = l;
    } else if (!split) {
        type = D_FEN;
    } else {
        type = l == nobs ? D_FENP : l == nobs + 1 ? D_FENM : l == nobs + 2 ? D_VB : D_WB;
    }
}

__device__ __forceinline__ void dd_bounds(const KP& P, int type, double& cl, double& cu)
{
    switch (type) {
    case D_CIR:
    case D_ELP: cl = 0.0; cu = INFINITY; break;
    case D_FENP:
    case D_FENM: cl = -INFINITY; cu = P.bvx_hi; break;
    case D_FEN:
    case D_VB: cl = P.bvx_lo; cu = P.bvx_hi; break;
    case D_WB: cl = -P.dth; cu = P.dth; break;
    default: cl = -INFINITY; cu = INFINITY;
    }
}

// state lanes k = 0..N roll the unicycle out from x0 with decision U (LDS) into ST
template <int N>
__device__ void dd_rollout(const double* cst, const double* U, double* ST, int lane)
{
    const double T = cst[DK_T];
    double th = cst[DK_X2];
#pragma unroll
    for (int j = 0; j < N; ++j) th += j < lane ? U[2 * j + 1] : 0.0;
    double sn, cs;
    sincos(th, &sn, &cs);
    const double tc = T * cs, ts = T * sn;
    const double v = lane < N ? U[2 * (lane < N ? lane : 0)] : 0.0;
    const double ax = tc * v, ay = ts * v;
    double px = cst[DK_X0], py = cst[DK_X1];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const double a = bcast(ax, j), b = bcast(ay, j);
        px += j < lane ? a : 0.0;
        py += j < lane ? b : 0.0;
    }
    if (lane <= N) {
        double* s = ST + DD_ST * lane;
        s[0] = px; s[1] = py; s[2] = th; s[3] = tc; s[4] = ts;
    }
}

// column j pair (v_j, w_j) of d(px, py)_k / du for a lane-varying step k (rows of cal_dx_du :534-566):
//   d px_k / d v_j = T cos th_j,  d py_k / d v_j = T sin th_j,  d px_k / d w_j = -(py_k - py_{j+1}),
//   d py_k / d w_j = px_k - px_{j+1},  d th_k / d w_j = 1   (all for j < k, else 0)
struct DDCol {
    double xv, yv, xw, yw, tw;
};
__device__ __forceinline__ DDCol dd_col(const double* ST, int j, int k, double pxk, double pyk)
{
    const double* s = ST + DD_ST * j;
    const double* s1 = ST + DD_ST * (j + 1);
    const bool in = j < k;
    DDCol c;
    c.xv = in ? s[3] : 0.0;
    c.yv = in ? s[4] : 0.0;
    c.xw = in ? -(pyk - s1[1]) : 0.0;
    c.yw = in ? (pxk - s1[0]) : 0.0;
    c.tw = in ? 1.0 : 0.0;
    return c;
}

// value of DD row `type` at (ST, U); JAC: its Jacobian row is written to Jout[0..n-1] (OBJ rows also
// return their local Hessian parts in hx)
template <int N, bool JAC>
__device__ double dd_row(int type, int k, const double (&o)[6], const double* cst, const double* ST,
                         const double* U, double* Jout, double (&hx)[8])
{
    constexpr int n = 2 * N;
    const double gm1 = cst[DK_GM1], sfen = cst[DK_S];
    double c = 0.0;
    if (type == D_CIR || type == D_ELP) {
        const double* s1 = ST + DD_ST * (k + 1);
        const double* s0 = ST + DD_ST * k;
        const double x1 = s1[0] - o[0], y1 = s1[1] - o[1], x0 = s0[0] - o[0], y0 = s0[1] - o[1];
        c = (o[2] * x1 * x1 + o[3] * x1 * y1 + o[4] * y1 * y1 - o[5]) +
            gm1 * (o[2] * x0 * x0 + o[3] * x0 * y0 + o[4] * y0 * y0 - o[5]);
        if (JAC) {
            const double g1x = 2 * o[2] * x1 + o[3] * y1, g1y = 2 * o[4] * y1 + o[3] * x1;
            const double g0x = gm1 * (2 * o[2] * x0 + o[3] * y0), g0y = gm1 * (2 * o[4] * y0 + o[3] * x0);
#pragma unroll
            for (int j = 0; j < N; ++j) {
                const DDCol a1 = dd_col(ST, j, k + 1, s1[0], s1[1]);
                const DDCol a0 = dd_col(ST, j, k, s0[0], s0[1]);
                Jout[2 * j] = g1x * a1.xv + g1y * a1.yv + g0x * a0.xv + g0y * a0.yv;
                Jout[2 * j + 1] = g1x * a1.xw + g1y * a1.yw + g0x * a0.xw + g0y * a0.yw;
            }
        }
    } else if (type == D_OBJ) {
        const double* sk = ST + DD_ST * k;
        const double w = cst[DK_Q] + (k == 1 ? cst[DK_P] : 0.0), r = cst[DK_R], t = cst[DK_TT];
        const double dxg = cst[DK_GX] - sk[0], dyg = cst[DK_GY] - sk[1];
        const double phi = sk[2] - atan2(dyg, dxg);
        const double up0 = k >= 2 ? U[2 * k - 4] : cst[DK_LU0], up1 = k >= 2 ? U[2 * k - 3] : cst[DK_LU1];
        const double d0 = U[2 * k - 2] - up0, d1 = U[2 * k - 1] - up1;
        c = w * (dxg * dxg + dyg * dyg) + r * phi * phi + t * (d0 * d0 + d1 * d1);
        if (JAC) {
            const double rho2 = dxg * dxg + dyg * dyg, ir2 = rho2 > 0.0 ? 1.0 / rho2 : 0.0;   // (§2 item 7)
            const double gp0 = -dyg * ir2, gp1 = dxg * ir2;
            const double ax = -2 * w * dxg + 2 * r * phi * gp0, ay = -2 * w * dyg + 2 * r * phi * gp1, at = 2 * r * phi;
#pragma unroll
            for (int j = 0; j < N; ++j) {
                const DDCol a = dd_col(ST, j, k, sk[0], sk[1]);
                const double sm = j == k - 1 ? 2 * t : (j == k - 2 ? -2 * t : 0.0);
                Jout[2 * j] = ax * a.xv + ay * a.yv + sm * d0;
                Jout[2 * j + 1] = ax * a.xw + ay * a.yw + at * a.tw + sm * d1;
            }
            const double ir4 = ir2 * ir2;
            const double s00 = 2 * dxg * dyg * ir4, s01 = (dyg * dyg - dxg * dxg) * ir4, s11 = -2 * dxg * dyg * ir4;
            hx[0] = 2 * w + 2 * r * (gp0 * gp0 - phi * s00);
            hx[1] = 2 * r * (gp0 * gp1 - phi * s01);
            hx[2] = 2 * w + 2 * r * (gp1 * gp1 - phi * s11);
            hx[3] = 2 * r * gp0;
            hx[4] = 2 * r * gp1;
            hx[5] = 2 * r;
            hx[6] = ax;
            hx[7] = ay;
        }
    } else if (type != D_NONE) {
        const double v = U[2 * k], wv = U[2 * k + 1];
        double jv = 1.0, jw = 0.0;
        switch (type) {
        case D_FENP: c = v + sfen * wv; jw = sfen; break;
        case D_FENM: c = v - sfen * wv; jw = -sfen; break;
        case D_VB: c = v; break;
        case D_WB: c = wv; jv = 0.0; jw = 1.0; break;
        case D_FEN: c = sfen * fabs(wv) + v; jw = sfen * (wv == 0.0 ? 0.0 : copysign(1.0, wv)); break;   // den_du
        default: break;
        }
        if (JAC) {
#pragma unroll
            for (int a = 0; a < n; ++a) Jout[a] = a == 2 * k ? jv : (a == 2 * k + 1 ? jw : 0.0);
        }
    } else if (JAC) {
#pragma unroll
        for (int a = 0; a < n; ++a) Jout[a] = 0.0;
    }
    return c;
}

// DD prologue: inputs, obstacle forms, constants; returns the number of valid circles / ellipses
template <int N>
__device__ void dd_prologue(const KP& P, const DDW<N>& w, long long b, int lane, int nc_max, int ne_max, int& ncv,
                            int& nev)
{
    constexpr int n = 2 * N;
    const double* x0 = P.x0 + 3 * b;
    ncv = min(P.nc[b], nc_max);
    nev = P.ne ? min(P.ne[b], ne_max) : 0;
    const int nobs = nc_max + ne_max;
    for (int j = lane; j <= nobs; j += WAVE) {
        double o[6] = {0, 0, 0, 0, 0, 0};
        if (j < nc_max) {
            if (j < ncv) {
                const double* c = P.cir + ((size_t)b * nc_max + j) * 3;
                o[0] = c[0]; o[1] = c[1]; o[2] = 1.0; o[4] = 1.0; o[5] = c[2] * c[2];
            }
        } else if (j < nobs) {
            const int e = j - nc_max;
            if (e < nev) {
                const double* el = P.elp + ((size_t)b * ne_max + e) * 5;
                double se, ce;
                sincos(el[4], &se, &ce);
                o[0] = el[0]; o[1] = el[1];
                o[2] = (el[3] * ce) * (el[3] * ce) + (el[2] * se) * (el[2] * se);
                o[3] = 2 * ce * se * (el[3] * el[3] - el[2] * el[2]);
                o[4] = (el[3] * se) * (el[3] * se) + (el[2] * ce) * (el[2] * ce);
                o[5] = (el[3] * el[2]) * (el[3] * el[2]);
            }
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) w.obs6[6 * j + i] = o[i];
    }
    if (lane == 0) {
        w.cst[DK_GM1] = P.gm1; w.cst[DK_S] = P.s; w.cst[DK_Q] = P.q; w.cst[DK_P] = P.p; w.cst[DK_R] = P.r;
        w.cst[DK_GX] = P.goal[2 * b]; w.cst[DK_GY] = P.goal[2 * b + 1]; w.cst[DK_T] = P.dt; w.cst[DK_TT] = P.dd_t;
        w.cst[DK_LU0] = P.last_u ? P.last_u[2 * b] : 0.0; w.cst[DK_LU1] = P.last_u ? P.last_u[2 * b + 1] : 0.0;
        w.cst[DK_TOL] = P.tol; w.cst[DK_ACCTOL] = P.acc_tol;
        w.cst[DK_X0] = x0[0]; w.cst[DK_X1] = x0[1]; w.cst[DK_X2] = x0[2];
    }
    if (lane < 16) w.Ua[lane] = lane < n ? P.u0[(size_t)b * n + lane] : 0.0;
    wave_sync();
}

// Hessian parts per step k (lane k = 1..N): objective parts from the OBJ rows + D-CBF rows of steps k-1
// (post-step state) and k (pre-step state, gamma - 1 factor)
template <int N>
__device__ void dd_hess_steps(const DDW<N>& w, const double* ST, int lane, int rps, int nobs)
{
    if (lane < 1 || lane > N) return;
    const int k = lane;
    const double* ho = w.hobj + 8 * k;
    double h00 = ho[0], h01 = ho[1], h11 = ho[2], h02 = ho[3], h12 = ho[4], h22 = ho[5], g0 = ho[6], g1 = ho[7];
    const double px = ST[DD_ST * k], py = ST[DD_ST * k + 1], gm1 = w.cst[DK_GM1];
#pragma unroll 4
    for (int j = 0; j < nobs; ++j) {
        const double* o = w.obs6 + 6 * j;
        const double x = px - o[0], y = py - o[1];
        const double dx = 2 * o[2] * x + o[3] * y, dy = 2 * o[4] * y + o[3] * x;
        double y1 = w.ry[(k - 1) * rps + j];
        double y0 = k < N ? w.ry[k * rps + j] * gm1 : 0.0;
        const double yy = y1 + y0;
        h00 -= yy * 2 * o[2];
        h01 -= yy * o[3];
        h11 -= yy * 2 * o[4];
        g0 -= yy * dx;
        g1 -= yy * dy;
    }
    double* hl = w.hl + 8 * k;
    hl[0] = h00; hl[1] = h01; hl[2] = h11; hl[3] = h02; hl[4] = h12; hl[5] = h22; hl[6] = g0; hl[7] = g1;
}

// exact Hessian entry H[a][b] (rollout second derivatives included) + smoothness term
template <int N>
__device__ double dd_hess_entry(const DDW<N>& w, const double* ST, int a, int b)
{
    const double T = w.cst[DK_T], t = w.cst[DK_TT];
    const int ja = a >> 1, jb = b >> 1;
    const bool va = (a & 1) == 0, vb = (b & 1) == 0;
    double h = 0.0;
#pragma unroll
    for (int k = 1; k <= N; ++k) {
        const double* sk = ST + DD_ST * k;
        const double* hl = w.hl + 8 * k;
        // d(px, py, th)_k / du_a and / du_b
        double xa, ya, ta, xb, yb, tb;
        {
            const double* s = ST + DD_ST * ja;
            const double* s1 = ST + DD_ST * (ja + 1);
            const bool in = ja < k;
            xa = in ? (va ? s[3] : -(sk[1] - s1[1])) : 0.0;
            ya = in ? (va ? s[4] : (sk[0] - s1[0])) : 0.0;
            ta = (in && !va) ? 1.0 : 0.0;
        }
        {
            const double* s = ST + DD_ST * jb;
            const double* s1 = ST + DD_ST * (jb + 1);
            const bool in = jb < k;
            xb = in ? (vb ? s[3] : -(sk[1] - s1[1])) : 0.0;
            yb = in ? (vb ? s[4] : (sk[0] - s1[0])) : 0.0;
            tb = (in && !vb) ? 1.0 : 0.0;
        }
        h += xa * (hl[0] * xb + hl[1] * yb + hl[3] * tb) + ya * (hl[1] * xb + hl[2] * yb + hl[4] * tb) +
             ta * (hl[3] * xb + hl[4] * yb + hl[5] * tb);
        // second derivatives of px_k, py_k
        double sxx = 0.0, syy = 0.0;
        if (va != vb) {
            const int jv = va ? ja : jb, jw = va ? jb : ja;   // d2 / dv_jv dw_jw, jw < jv < k
            if (jw < jv && jv < k) {
                sxx = -ST[DD_ST * jv + 4];
                syy = ST[DD_ST * jv + 3];
            }
        } else if (!va) {
            const int mm = ja > jb ? ja : jb;
            if (mm < k) {
                sxx = -(sk[0] - ST[DD_ST * (mm + 1)]);
                syy = -(sk[1] - ST[DD_ST * (mm + 1) + 1]);
            }
        }
        h += hl[6] * sxx + hl[7] * syy;
    }
    if (a == b) h += 2 * t * (ja < N - 1 ? 2.0 : 1.0);
    if ((a & 1) == (b & 1) && (ja - jb == 1 || jb - ja == 1)) h -= 2 * t;
    return h;
}

// ------------------------------------------------------------------------------------------------
// DD solve kernel (one instance per wave); RPL row groups of 64 lanes, KSM = 16 RPL J-layout steps
// ------------------------------------------------------------------------------------------------
// DD solve kernels: 2 waves per SIMD (256 VGPRs).  At 4 waves they spilled 132 / 244 / 356 B per lane
// (RPL = 1 / 2 / 3); at 2 waves: N = 3, 5 circles +11 %, N = 5, 5 + 5 obstacles 2.0x
// (profiles/r1f/ab_dd_occupancy.log)
#ifndef ALIP_DD_WAVES_RPL1
#define ALIP_DD_WAVES_RPL1 2
#endif
#ifndef ALIP_DD_WAVES_RPL2
#define ALIP_DD_WAVES_RPL2 2
#endif
template <int RPL>
constexpr int dd_solve_waves() { return RPL > 1 ? ALIP_DD_WAVES_RPL2 : ALIP_DD_WAVES_RPL1; }

template <int N, int RPL>
__global__ __launch_bounds__(256, dd_solve_waves<RPL>()) void dd_solve_kernel(KP Pv)
{
    constexpr int n = 2 * N;
    constexpr int KSM = 16 * RPL;
    constexpr int KLD = 17;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    KP* Ps = reinterpret_cast<KP*>(smem);
    double* wsb = smem + KP_DOUBLES;
    if (threadIdx.x == 0) *Ps = Pv;
    __syncthreads();
    const KP& P = *Ps;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
    int lane = lane_id();
    const long long b = (long long)blockIdx.x * WAVES_PER_BLOCK + wv;
    if (b >= P.B) return;
    if (P.active && !P.active[b]) return;   // rollout: instance already at its goal
    const int mr4 = rfl(P.mr4), mo4 = rfl(P.mo4), m_max = rfl(P.m_max), rps = rfl(P.rps);
    const int nc_max = rfl(P.nc_max), ne_max = rfl(P.ne_max), nobs = nc_max + ne_max, max_iter = rfl(P.max_iter);
    DDW<N> w = carve_dd<N>(wsb + (size_t)wv * ddw_doubles<N>(nobs, mo4), nobs, mo4);
    int ncv, nev;
    dd_prologue<N>(P, w, b, lane, nc_max, ne_max, ncv, nev);
    double* ST = w.STa;   // current point
    double* STt = w.STb;  // trial point
    double* U = w.Ua;
    double* Ut = w.Ub;
    dd_rollout<N>(w.cst, U, ST, lane);
    for (int i = lane; i < 16 * mo4; i += WAVE) w.Jd[i] = 0.0;
    wave_sync();
    int g4 = lane >> 4, col = lane & 15;
#define HL(q) (cl[q] != -INFINITY)
#define HU(q) (cu[q] != INFINITY)
#define RELANE()                           \
    do {                                   \
        RELAUNDER(lane);                   \
        g4 = lane >> 4;                    \
        col = lane & 15;                   \
        for (int q_ = 0; q_ < RPL; ++q_) { \
            RELAUNDER(rtype[q_]);          \
            RELAUNDER(rk[q_]);             \
            RELAUNDER(roi[q_]);            \
            RELAUNDER(cl[q_]);             \
            RELAUNDER(cu[q_]);             \
        }                                  \
    } while (0)
    int rtype[RPL], rk[RPL], roi[RPL];
    double cl[RPL], cu[RPL], cr[RPL], sr[RPL], zl[RPL], zu[RPL], idl[RPL], idu[RPL];
    double mu = uni(P.mu_init);
    double th0 = 0.0, nbl = 0.0, mal = 0.0, fo = 0.0, lg0 = 0.0;
    double hx[8];
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
        const int r = lane + WAVE * q;
        int t, k, oi;
        dd_decode(r, rps, m_max, nc_max, ne_max, ncv, nev, true, t, k, oi);
        if (r >= mr4 && r < mr4 + N) {
            t = D_OBJ;
            k = r - mr4 + 1;
        }
        rtype[q] = t;
        rk[q] = k;
        roi[q] = oi;
        double clo, cuo;
        dd_bounds(P, t, clo, cuo);
        if (r < mr4) {
            w.rclo[r] = clo;
            w.rcuo[r] = cuo;
        }
        nbl += (double)isfinite(clo) + (double)isfinite(cuo);
        mal += t < D_NONE ? 1.0 : 0.0;
        cl[q] = isfinite(clo) ? clo - 1e-8 * fmax(1.0, fabs(clo)) : -INFINITY;
        cu[q] = isfinite(cuo) ? cuo + 1e-8 * fmax(1.0, fabs(cuo)) : INFINITY;
        double o[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) o[i] = w.obs6[6 * oi + i];
        cr[q] = dd_row<N, false>(t, k, o, w.cst, ST, U, nullptr, hx);
        double v = cr[q];
        const double pl = HL(q) ? fmin(1e-2 * fmax(1.0, fabs(cl[q])), 1e-2 * (cu[q] - cl[q])) : 0.0;
        const double pu = HU(q) ? fmin(1e-2 * fmax(1.0, fabs(cu[q])), 1e-2 * (cu[q] - cl[q])) : 0.0;
        if (HL(q) && HU(q))
            v = fmin(fmax(v, cl[q] + pl), cu[q] - pu);
        else if (HL(q))
            v = fmax(v, cl[q] + pl);
        else if (HU(q))
            v = fmin(v, cu[q] - pu);
        sr[q] = t < D_NONE ? v : 0.0;
        zl[q] = HL(q) ? 1.0 : 0.0;
        zu[q] = HU(q) ? 1.0 : 0.0;
        const double dl = sr[q] - cl[q], du = cu[q] - sr[q];
        idl[q] = HL(q) ? rcp_nr(dl) : 0.0;
        idu[q] = HU(q) ? rcp_nr(du) : 0.0;
        lg0 += HL(q) ? (HU(q) ? log(dl * du) : log(dl)) : (HU(q) ? log(du) : 0.0);
        if (t < D_NONE) th0 += fabs(cr[q] - sr[q]);
        if (t == D_OBJ) fo += cr[q];
    }
    // IPOPT's default NLP scaling at the starting point (MPC_DD_sig_step.py:176-190 sets no scaling option): the
    // objective's gradient in u (the OBJ rows' Jacobian rows), the objective scaled by 100 / max |grad f| where that
    // exceeds 100 — all four weights, the objective being linear in them
    {
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int r = lane + WAVE * q;
            if (rtype[q] == D_OBJ) {
                double o[6] = {0, 0, 0, 0, 0, 0}, hxs[8];
                (void)dd_row<N, true>(D_OBJ, rk[q], o, w.cst, ST, U, w.Jd + 16 * r, hxs);
            }
        }
        wave_sync();
        double gu = 0.0;
        if (lane < n) {
#pragma unroll
            for (int k = 0; k < N; ++k) gu += w.Jd[16 * (mr4 + k) + lane];
        }
        const double gm = wmax(fabs(gu));
        const double dfo = uni(gm > 100.0 ? fmax(1e-8, 100.0 / gm) : 1.0);
        wave_sync();
        if (dfo != 1.0) {
            if (lane == 0) {
                w.cst[DK_Q] *= dfo;
                w.cst[DK_P] *= dfo;
                w.cst[DK_R] *= dfo;
                w.cst[DK_TT] *= dfo;
            }
            fo *= dfo;
#pragma unroll
            for (int q = 0; q < RPL; ++q)
                if (rtype[q] == D_OBJ) cr[q] *= dfo;
            wave_sync();
        }
    }
    wsum2(th0, nbl);
    wsum2(fo, lg0);
    mal = wsum(mal);
    double f_cur = fo, lsum_cur = lg0;
    if (lane == 0) {
        w.cst[DK_THMAX] = 1e4 * fmax(1.0, th0);
        w.cst[DK_THMIN] = 1e-4 * fmax(1.0, th0);
        w.cst[DK_MACT] = mal;
        w.cst[DK_NBL] = nbl;
    }
    wave_sync();
    double fth0 = INFINITY, fph0 = INFINITY, fth1 = INFINITY, fph1 = INFINITY;
    int nf = 0;
    double dw_last = 0.0;
    int status = -1, it = 0, n_rest = 0;
    double e0 = INFINITY;
    const double gth = 1e-5, gph = 1e-8, sth = 1.1, sph = 2.3, eta = 1e-8, gal = 0.05;

    for (it = 0; it <= max_iter; ++it) {
        // ---- row layout: Jacobian rows at the current point (OBJ rows: grad f_k + Hessian parts)
        RELANE();
        bool at_goal = false;   // an OBJ row's state exactly on the goal (cfg.goal_singular)
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int r = lane + WAVE * q;
            double o[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) o[i] = w.obs6[6 * roi[q] + i];
            // every lane owns a row (mo4 = 64 RPL); columns n..15 stay zero (zeroed in the prologue)
            dd_row<N, true>(rtype[q], rk[q], o, w.cst, ST, U, w.Jd + 16 * r, hx);
            w.ry[r] = rtype[q] == D_OBJ ? -1.0 : zl[q] - zu[q];
            if (rtype[q] == D_OBJ) {
#pragma unroll
                for (int i = 0; i < 8; ++i) w.hobj[8 * rk[q] + i] = hx[i];
                const double* sk = ST + DD_ST * rk[q];
                const double dxg = w.cst[DK_GX] - sk[0], dyg = w.cst[DK_GY] - sk[1];
                at_goal |= dxg * dxg + dyg * dyg == 0.0;
            }
        }
        wave_sync();
        // ---- J layout: gl = J^T y - grad f
        RELANE();
        double gl = 0.0;
#pragma unroll
        for (int s = 0; s < KSM; ++s) {
            const int r = 4 * s + g4;
            gl += w.Jd[16 * r + col] * w.ry[r];
        }
        gl = gsum(gl);
        // ---- convergence test and barrier update
        double ru = (g4 == 0 && col < n) ? fabs(gl) : 0.0;
        double rcm = 0.0, nz = 0.0, comp0 = 0.0;
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const double dl = sr[q] - cl[q], du = cu[q] - sr[q];
            if (rtype[q] < D_NONE) rcm = fmax(rcm, fabs(cr[q] - sr[q]));
            nz += fabs(zl[q]) + fabs(zu[q]);
            if (HL(q)) comp0 = fmax(comp0, fabs(dl * zl[q]));
            if (HU(q)) comp0 = fmax(comp0, fabs(du * zu[q]));
        }
        ru = wmax(ru);
        rcm = wmax(rcm);
        nz = wsum(nz);
        comp0 = wmax(comp0);
        const double sd = uni(fmax(100.0, nz / (w.cst[DK_MACT] + n)) / 100.0);
        const double sc = uni(fmax(100.0, nz / fmax(1.0, w.cst[DK_NBL])) / 100.0);
        const double base_err = uni(fmax(ru / sd, rcm));
        e0 = uni(fmax(base_err, comp0 / sc));
        // cfg.goal_singular = ABORT (MPC_DD_sig_step.py:527-531 divides 0 by 0 here): Invalid_Number_Detected
        if (rfl(P.goal_abort) && __ballot(at_goal) != 0ull) {
            status = -13;
            break;
        }
        if (e0 <= w.cst[DK_TOL]) {
            status = 0;
            break;
        }
        if (it == max_iter) break;
        {
            const double mu_min = w.cst[DK_TOL] / 11.0;   // (IPOPT's floor, as solve_kernel)
            const double mu_prev = mu;
            for (int t = 0; t < 8; ++t) {
                double cm = 0.0;
#pragma unroll
                for (int q = 0; q < RPL; ++q) {
                    const double dl = sr[q] - cl[q], du = cu[q] - sr[q];
                    if (HL(q)) cm = fmax(cm, fabs(dl * zl[q] - mu));
                    if (HU(q)) cm = fmax(cm, fabs(du * zu[q] - mu));
                }
                cm = wmax(cm);
                if (fmax(base_err, cm / sc) <= 10.0 * mu && mu > mu_min)
                    mu = uni(fmax(mu_min, fmin(0.2 * mu, mu * sqrt(mu))));
                else
                    break;
            }
            if (mu != mu_prev) nf = 0;
        }
        const double tau = uni(fmax(0.99, 1.0 - mu));
        // ---- Sigma, rhs weights, Hessian parts
        RELANE();
        double rcv[RPL];
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int r = lane + WAVE * q;
            const double sg = zl[q] * idl[q] + zu[q] * idu[q];
            rcv[q] = rtype[q] < D_NONE ? cr[q] - sr[q] : 0.0;
            double wr = mu * idl[q] - mu * idu[q] - sg * rcv[q];
            wr = rtype[q] == D_OBJ ? -1.0 : wr;
            if (r < mo4) {
                w.rsig[r] = sg;
                w.rw[r] = wr;
            }
        }
        dd_hess_steps<N>(w, ST, lane, rps, nobs);
        wave_sync();
        // ---- K = J^T Sigma J (MFMA) + exact Hessian, rhs = J^T w - grad f
        RELANE();
        double rhs;
        {
            d4 acc0 = d4{0.0, 0.0, 0.0, 0.0}, acc1 = d4{0.0, 0.0, 0.0, 0.0};
            double pw = 0.0;
#pragma unroll
            for (int s = 0; s < KSM; ++s) {
                const int r = 4 * s + g4;
                const double j = w.Jd[16 * r + col];
                const double sg = w.rsig[r];
                pw += j * w.rw[r];
                if (s & 1)
                    acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(j, sg * j, acc1, 0, 0, 0);
                else
                    acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(j, sg * j, acc0, 0, 0, 0);
            }
            rhs = gsum(pw);
#pragma unroll
            for (int i = 0; i < 4; ++i) w.K[(g4 + 4 * i) * KLD + col] = acc0[i] + acc1[i];
        }
        wave_sync();
        for (int e = lane; e < n * n; e += WAVE) {
            const int a = e / n, bb = e - a * n;
            w.K[a * KLD + bb] += dd_hess_entry<N>(w, ST, a, bb);
        }
        wave_sync();
        // ---- factor with inertia correction, solve for du
        RELANE();
        double xv;
        bool fact_ok = true;
        {
            const double rhs_l = lane < n ? rhs : 0.0;
            double a[n];
            double myidg = 1.0;
#pragma unroll
            for (int j = 0; j < n; ++j) a[j] = lane < n ? w.K[lane * KLD + j] : (lane == j ? 1.0 : 0.0);
            if (!chol_rows<n>(a, myidg, lane)) {
                double dw = dw_last == 0.0 ? 1e-4 : fmax(1e-20, dw_last / 3.0);
                for (;;) {
#pragma unroll
                    for (int j = 0; j < n; ++j)
                        a[j] = (lane < n ? w.K[lane * KLD + j] : (lane == j ? 1.0 : 0.0)) + (lane == j ? dw : 0.0);
                    if (chol_rows<n>(a, myidg, lane)) break;
                    dw *= dw_last == 0.0 ? 100.0 : 8.0;
                    if (dw > 1e40) {   // (not IPOPT's 1e20)
                        fact_ok = false;
                        break;
                    }
                }
                dw_last = uni(dw);
            }
            double acc = 0.0, yv = 0.0;
#pragma unroll
            for (int k = 0; k < n; ++k) {
                const double yk = bcast((rhs_l - acc) * myidg, k);
                yv = lane == k ? yk : yv;
                acc += lane > k ? a[k] * yk : 0.0;
            }
            wave_sync();
            if (lane < n) {
#pragma unroll
                for (int j = 0; j < n; ++j) w.K[lane * KLD + j] = j <= lane ? a[j] : 0.0;
            }
            wave_sync();
            acc = 0.0;
            xv = 0.0;
#pragma unroll
            for (int i = n - 1; i >= 0; --i) {
                const double xi = bcast((yv - acc) * myidg, i);
                xv = lane == i ? xi : xv;
                acc += lane < i ? w.K[i * KLD + (lane & 15)] * xi : 0.0;
            }
        }
        if (lane < 16) w.dU[lane] = lane < n ? xv : 0.0;
        wave_sync();
        if (!fact_ok) {
            status = -3;
            break;
        }
        // ---- slack / multiplier steps, fraction to boundary
        RELANE();
        double dS[RPL], dZl[RPL], dZu[RPL];
        double ap = 1.0, az = 1.0, theta = 0.0, sl = 0.0, gdv = 0.0;
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int r = lane + WAVE * q;
            double jd = 0.0;
            if (r < mo4) {
#pragma unroll
                for (int a = 0; a < n; ++a) jd += w.Jd[16 * r + a] * w.dU[a];
            }
            if (rtype[q] == D_OBJ) gdv += jd;
            dS[q] = rtype[q] < D_NONE ? jd + rcv[q] : 0.0;
            dZl[q] = HL(q) ? mu * idl[q] - zl[q] - zl[q] * idl[q] * dS[q] : 0.0;
            dZu[q] = HU(q) ? mu * idu[q] - zu[q] + zu[q] * idu[q] * dS[q] : 0.0;
            const double dl = sr[q] - cl[q], du = cu[q] - sr[q];
            const double ids = rcp_nr(dS[q]);
            if (HL(q) && dS[q] < 0) ap = fmin(ap, -tau * dl * ids);
            if (HU(q) && dS[q] > 0) ap = fmin(ap, tau * du * ids);
            if (HL(q) && dZl[q] < 0) az = fmin(az, -tau * zl[q] * rcp_nr(dZl[q]));
            if (HU(q) && dZu[q] < 0) az = fmin(az, -tau * zu[q] * rcp_nr(dZu[q]));
            theta += fabs(rcv[q]);
            sl += (HL(q) ? dS[q] * idl[q] : 0.0) - (HU(q) ? dS[q] * idu[q] : 0.0);
        }
        ap = wmin(ap);
        az = wmin(az);
        wsum2(theta, gdv);
        sl = wsum(sl);
        const double phi = uni(f_cur - mu * lsum_cur);
        const double gphi = uni(gdv - mu * sl);
        const double lsw = uni(gphi < 0 ? sth * log(theta) - sph * log(-gphi) : 0.0);
        double amin;
        if (gphi < 0) {
            amin = fmin(gth, gph * theta / -gphi);
            if (theta <= w.cst[DK_THMIN]) amin = fmin(amin, exp(lsw));
        } else {
            amin = gth;
        }
        amin *= gal;
        amin = uni(amin > 0.0 ? amin : 8.673617379884035e-19);   // (floor where the formula gives 0: DESIGN.md §2 item 8)
        // ---- filter line search: trial u = U + a dU, rolled out
        double a = ap;
        double la = uni(log(ap));
        bool accepted = false, ftype = false;
        double ctr[RPL];
        double ft = 0.0, lgt = 0.0;
        while (a >= amin) {
            RELANE();
            if (lane < 16) Ut[lane] = fma(a, w.dU[lane], U[lane]);
            wave_sync();
            dd_rollout<N>(w.cst, Ut, STt, lane);
            wave_sync();
            double tht = 0.0;
            ft = 0.0;
            lgt = 0.0;
            bool bad = false;
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                double o[6];
#pragma unroll
                for (int i = 0; i < 6; ++i) o[i] = w.obs6[6 * roi[q] + i];
                ctr[q] = dd_row<N, false>(rtype[q], rk[q], o, w.cst, STt, Ut, nullptr, hx);
                const double st = sr[q] + a * dS[q];
                if (rtype[q] < D_NONE) tht += fabs(ctr[q] - st);
                if (rtype[q] == D_OBJ) ft += ctr[q];
                const double d1 = st - cl[q], d2 = cu[q] - st;
                if (HL(q) && !(d1 > 0)) bad = true;
                if (HU(q) && !(d2 > 0)) bad = true;
                lgt += HL(q) ? (HU(q) ? log(d1 * d2) : log(d1)) : (HU(q) ? log(d2) : 0.0);
            }
            wsum2(ft, tht);
            lgt = wsum(lgt);
            const bool anybad = __ballot(bad) != 0ull;
            const double pht = anybad ? INFINITY : ft - mu * lgt;
            bool ok = isfinite(pht) && tht < w.cst[DK_THMAX];
            if (ok) {
                const bool b0 = lane < nf && !(tht < fth0 || pht < fph0);
                const bool b1 = lane + WAVE < nf && !(tht < fth1 || pht < fph1);
                ok = __ballot(b0 || b1) == 0ull;
            }
            if (ok) {
                const bool switching = gphi < 0 && la > lsw;
                if (switching && theta <= w.cst[DK_THMIN]) {
                    if (pht <= phi + eta * a * gphi) {
                        accepted = true;
                        ftype = true;
                    }
                } else if (tht <= (1 - gth) * theta || pht <= phi - gph * theta) {
                    accepted = true;
                    ftype = false;
                }
            }
            if (accepted) break;
            a = uni(a * 0.5);
            la = uni(la - M_LN2);
        }
        RELANE();
        if (accepted) {
            if (!ftype && nf < FILTER_CAP) {
                const double fvt = (1 - gth) * theta, fvp = phi - gph * theta;
                if ((nf & (WAVE - 1)) == lane) {
                    if (nf < WAVE) {
                        fth0 = fvt;
                        fph0 = fvp;
                    } else {
                        fth1 = fvt;
                        fph1 = fvp;
                    }
                }
                nf++;
            }
            // the trial point becomes the current one (swap the table roles)
            double* t1 = ST; ST = STt; STt = t1;
            double* t2 = U; U = Ut; Ut = t2;
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                sr[q] += a * dS[q];
                cr[q] = ctr[q];
            }
            f_cur = ft;
            lsum_cur = lgt;
        } else {
            // restoration substitute: shortest tried step, slacks reset onto c(u), filter reset
            a = uni(fmax(a, amin));
            if (lane < 16) Ut[lane] = fma(a, w.dU[lane], U[lane]);
            wave_sync();
            dd_rollout<N>(w.cst, Ut, STt, lane);
            wave_sync();
            double* t1 = ST; ST = STt; STt = t1;
            double* t2 = U; U = Ut; Ut = t2;
            double fr = 0.0, lr = 0.0;
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                double o[6];
#pragma unroll
                for (int i = 0; i < 6; ++i) o[i] = w.obs6[6 * roi[q] + i];
                cr[q] = dd_row<N, false>(rtype[q], rk[q], o, w.cst, ST, U, nullptr, hx);
                double v = cr[q];
                const double pl = HL(q) ? fmin(1e-2 * fmax(1.0, fabs(cl[q])), 1e-2 * (cu[q] - cl[q])) : 0.0;
                const double pu = HU(q) ? fmin(1e-2 * fmax(1.0, fabs(cu[q])), 1e-2 * (cu[q] - cl[q])) : 0.0;
                if (HL(q) && HU(q))
                    v = fmin(fmax(v, cl[q] + pl), cu[q] - pu);
                else if (HL(q))
                    v = fmax(v, cl[q] + pl);
                else if (HU(q))
                    v = fmin(v, cu[q] - pu);
                sr[q] = rtype[q] < D_NONE ? v : 0.0;
                const double d1 = sr[q] - cl[q], d2 = cu[q] - sr[q];
                lr += HL(q) ? (HU(q) ? log(d1 * d2) : log(d1)) : (HU(q) ? log(d2) : 0.0);
                if (rtype[q] == D_OBJ) fr += cr[q];
            }
            wsum2(fr, lr);
            f_cur = fr;
            lsum_cur = lr;
            nf = 0;
            n_rest++;
            double viol = 0.0;
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                const int r = lane + WAVE * q;
                if (r < mr4 && rtype[q] < D_NONE) {
                    if (HL(q)) viol = fmax(viol, w.rclo[r] - cr[q]);
                    if (HU(q)) viol = fmax(viol, cr[q] - w.rcuo[r]);
                }
            }
            viol = wmax(viol);
            if (n_rest >= REST_FAIL && viol > 1e-4) {
                status = 2;
                it++;
                break;
            }
        }
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            zl[q] += az * dZl[q];
            zu[q] += az * dZu[q];
            const double d1 = sr[q] - cl[q], d2 = cu[q] - sr[q];
            idl[q] = HL(q) ? rcp_nr(d1) : 0.0;
            idu[q] = HU(q) ? rcp_nr(d2) : 0.0;
            zl[q] = HL(q) ? fmin(fmax(zl[q], mu * 1e-10 * idl[q]), 1e10 * mu * idl[q]) : 0.0;
            zu[q] = HU(q) ? fmin(fmax(zu[q], mu * 1e-10 * idu[q]), 1e10 * mu * idu[q]) : 0.0;
        }
        wave_sync();
    }
    // ---- status + outputs (split rows measure the reference's f_en violation exactly)
    wave_sync();
    RELANE();
    if (status != 0 && status != 2 && status != -3 && status != -13) {
        double viol = 0.0;
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int r = lane + WAVE * q;
            if (r < mr4 && rtype[q] < D_NONE) {
                if (HL(q)) viol = fmax(viol, w.rclo[r] - cr[q]);
                if (HU(q)) viol = fmax(viol, cr[q] - w.rcuo[r]);
            }
        }
        viol = wmax(viol);
        if (e0 <= w.cst[DK_ACCTOL])
            status = 1;
        else if (viol > 1e-4)
            status = 2;
    }
    if (lane < n) P.u_out[(size_t)b * n + lane] = U[lane];
    if (P.foot_out && lane < 3) P.foot_out[3 * b + lane] = lane < 2 ? U[lane] : 0.0;
    if (P.x_pred && lane < 3 * N) P.x_pred[(size_t)b * 3 * N + lane] = ST[DD_ST * (lane / 3 + 1) + lane % 3];
    if (lane == 0) {
        if (P.status) P.status[b] = status;
        if (P.iters) P.iters[b] = it;
    }
#undef RELANE
#undef HL
#undef HU
}

// DD eval kernel: the reference callbacks (f, grad f, c, J, cl, cu, row activity) at given u, padded
// layout [circle slots, ellipse slots, f_en] per step
template <int N>
__global__ __launch_bounds__(256, 4) void dd_eval_kernel(KP Pv)
{
    constexpr int n = 2 * N;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    KP* Ps = reinterpret_cast<KP*>(smem);
    double* wsb = smem + KP_DOUBLES;
    if (threadIdx.x == 0) *Ps = Pv;
    __syncthreads();
    const KP& P = *Ps;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
    const int lane = lane_id();
    const long long b = (long long)blockIdx.x * WAVES_PER_BLOCK + wv;
    if (b >= P.B) return;
    const int mo4 = rfl(P.mo4), m_max = rfl(P.m_max), rps = rfl(P.rps);
    const int nc_max = rfl(P.nc_max), ne_max = rfl(P.ne_max), nobs = nc_max + ne_max;
    DDW<N> w = carve_dd<N>(wsb + (size_t)wv * ddw_doubles<N>(nobs, mo4), nobs, mo4);
    int ncv, nev;
    dd_prologue<N>(P, w, b, lane, nc_max, ne_max, ncv, nev);
    dd_rollout<N>(w.cst, w.Ua, w.STa, lane);
    wave_sync();
    const size_t mm = (size_t)m_max;
    double fk = 0.0, hx[8];
    for (int r = lane; r < m_max + N; r += WAVE) {
        int t, k, oi;
        if (r < m_max) {
            dd_decode(r, rps, m_max, nc_max, ne_max, ncv, nev, false, t, k, oi);
        } else {
            t = D_OBJ;
            k = r - m_max + 1;
            oi = 0;
        }
        double o[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) o[i] = w.obs6[6 * oi + i];
        // OBJ rows: grad f_k into LDS scratch; constraint rows: J row straight to HBM (or scratch)
        double* jo = t == D_OBJ ? w.Jd + 16 * (r - m_max)
                                : (P.J_out ? P.J_out + (b * mm + r) * n : w.Jd + 16 * (N + (lane & 31)));   // junk scratch
        const double c = dd_row<N, true>(t, k, o, w.cst, w.STa, w.Ua, jo, hx);
        if (t == D_OBJ) {
            fk += c;
        } else {
            double clv, cuv;
            dd_bounds(P, t, clv, cuv);
            if (P.c_out) P.c_out[b * mm + r] = c;
            if (P.cl_out) P.cl_out[b * mm + r] = clv;
            if (P.cu_out) P.cu_out[b * mm + r] = cuv;
            if (P.active_out) P.active_out[b * mm + r] = t != D_NONE;
        }
    }
    const double f = wsum(fk);
    wave_sync();
    if (lane < n && P.grad_out) {
        double g = 0.0;
        for (int k = 0; k < N; ++k) g += w.Jd[16 * k + lane];
        P.grad_out[b * n + lane] = g;
    }
    if (lane == 0) {
        if (P.f_out) P.f_out[b] = f;
        if (P.goal_eff_out) {
            P.goal_eff_out[2 * b] = P.goal[2 * b];
            P.goal_eff_out[2 * b + 1] = P.goal[2 * b + 1];
        }
    }
}

#if ALIP_PART_HOST
// ------------------------------------------------------------------------------------------------
// closed-loop rollout ("data_log replay" batch harness): after each solve, every
// active instance executes its first planned step on an ideal ALIP plant and re-plans from the touchdown
// state.  One thread per instance (HBM-bound, a few hundred bytes each):
//   x  <- x_pred[0]                 (= A x + B p_0; the continuous flow get_next_states over a full step,
//                                     MPC_LIP_modi.py:149-178, evaluated at t_rest = T)
//   u0 <- warm start from the plan  (modi: the previous x_mpc_tar unshifted, logger_mpc.py:325-331;
//                                    sig_step: [g2 .. gN, gN], MPC_LIP_sig_step.py:186-189; DD: previous
//                                    controls, last_u <- first control)
//   leg <- -leg                     (stance switch, main_sim_mpc.py:111)
//   close_2_goal: modi |pos_1 - goal| <= 0.15 (MPC_LIP_modi.py:108-115), sig_step any step <= 0.35
//   (MPC_LIP_sig_step.py:104-111), DD |pos_1 - goal| <= 0.35 (MPC_DD_sig_step.py:92-98); the episode
//   stops after that step (main_sim_mpc.py:121-131): the instance goes inactive.
// ------------------------------------------------------------------------------------------------
struct AdvP {
    long long B;
    int t, S, N, sd, n, variant;
    const double* goal;
    double* x;        // B x sd     (in/out)
    double* u0;       // B x n      (in/out)
    int8_t* leg;      // B          (in/out)
    double* last_u;   // B x 2      (in/out, DD)
    const double* u;  // B x n      solve outputs
    const double* foot;
    const double* x_pred;
    const int32_t* status;
    const int32_t* iters;
    uint8_t* active;  // B          (in/out)
    double* foot_traj;     // B x S x 3
    double* x_traj;        // B x (S+1) x sd
    int32_t* status_traj;  // B x S
    int32_t* iters_traj;   // B x S
    int32_t* steps_to_goal;  // B
    double* u_traj;        // B x S x n   the plan of every step (NaN after the goal)
};

__global__ __launch_bounds__(256) void advance_kernel(AdvP A)
{
    const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= A.B) return;
    const int t = A.t, S = A.S, sd = A.sd, n = A.n, N = A.N;
    if (!A.active[b]) {
        if (A.foot_traj)
            for (int i = 0; i < 3; ++i) A.foot_traj[((size_t)b * S + t) * 3 + i] = NAN;
        if (A.x_traj)
            for (int i = 0; i < sd; ++i) A.x_traj[((size_t)b * (S + 1) + t + 1) * sd + i] = A.x[(size_t)b * sd + i];
        if (A.status_traj) A.status_traj[(size_t)b * S + t] = ALIPMPC_ROLLOUT_DONE;
        if (A.iters_traj) A.iters_traj[(size_t)b * S + t] = 0;
        if (A.u_traj)
            for (int i = 0; i < n; ++i) A.u_traj[((size_t)b * S + t) * n + i] = NAN;
        return;
    }
    const double* xp = A.x_pred + (size_t)b * N * sd;
    if (A.foot_traj)
        for (int i = 0; i < 3; ++i) A.foot_traj[((size_t)b * S + t) * 3 + i] = A.foot[3 * b + i];
    if (A.status_traj) A.status_traj[(size_t)b * S + t] = A.status[b];
    if (A.iters_traj) A.iters_traj[(size_t)b * S + t] = A.iters[b];
    for (int i = 0; i < sd; ++i) {
        A.x[(size_t)b * sd + i] = xp[i];
        if (A.x_traj) A.x_traj[((size_t)b * (S + 1) + t + 1) * sd + i] = xp[i];
    }
    const double* ub = A.u + (size_t)b * n;
    double* u0 = A.u0 + (size_t)b * n;
    if (A.u_traj)
        for (int i = 0; i < n; ++i) A.u_traj[((size_t)b * S + t) * n + i] = ub[i];
    if (A.variant == ALIPMPC_VARIANT_SIG_STEP) {
        const int blk = n / N;
        for (int k = 0; k < N; ++k) {
            const int src = k + 1 < N ? k + 1 : N - 1;
            for (int i = 0; i < blk; ++i) u0[k * blk + i] = ub[src * blk + i];
        }
    } else {
        for (int i = 0; i < n; ++i) u0[i] = ub[i];
    }
    if (A.variant == ALIPMPC_VARIANT_DD) {
        A.last_u[2 * b] = ub[0];
        A.last_u[2 * b + 1] = ub[1];
    } else {
        A.leg[b] = (int8_t)(-A.leg[b]);
    }
    const double gx_ = A.goal[2 * b], gy_ = A.goal[2 * b + 1];
    bool close = false;
    const int kmax = A.variant == ALIPMPC_VARIANT_SIG_STEP ? N : 1;
    const double rad = A.variant == ALIPMPC_VARIANT_MODI ? 0.15 : 0.35;
    for (int k = 0; k < kmax; ++k) {
        const double dx = xp[k * sd] - gx_, dy = xp[k * sd + 1] - gy_;
        close = close || sqrt(dx * dx + dy * dy) <= rad;
    }
    if (close) {
        A.active[b] = 0;
        if (A.steps_to_goal) A.steps_to_goal[b] = t + 1;
    }
}

__global__ __launch_bounds__(256) void rollout_init_kernel(long long B, int S, int sd, const double* x0, double* xtraj,
                                                           uint8_t* active, int32_t* steps_to_goal)
{
    const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    active[b] = 1;
    if (steps_to_goal) steps_to_goal[b] = -1;
    if (xtraj)
        for (int i = 0; i < sd; ++i) xtraj[(size_t)b * (S + 1) * sd + i] = x0[(size_t)b * sd + i];
}

// ------------------------------------------------------------------------------------------------
// closed loop at the reference's control rate (alipmpc_closed_loop_batch): main_sim_mpc.py:41,65-135 driving
// Logger.set_stf_head / gen_nex_foot_input (data_procs/logger_mpc.py:270-371) on an ALIP plant.  Per tick
// i of step s (rest_t = T - i T / f_cyc):
//   cl_project_kernel  tick 0: set_stf_head (tube_func, avg_hd -> hd_input_pr, hd_input_cos);
//                      x_nex = get_next_states(plant, [stance foot, hd_input_pr], rest_t) (MPC_LIP_modi.py:149-178);
//                      warm start: [x_nex] x 3 on the first call, else the previous plan x_mpc_tar (unshifted,
//                      num_step >= 1 in the driver; sig_step: [g2..gN, gN] as solveMPCCBF does it)
//   solve launch       od_ev = -leg_ind
//   cl_update_kernel   nex_turn, mpc_hds_list, mpc_state_tar from the solve; the plant moves dt = T / f_cyc
//                      around the stance foot (+ an optional seeded velocity kick: plant mismatch); after the
//                      last tick: touchdown, stance foot <- p_list[0][0:2] of that solve, leg_ind <- -leg_ind,
//                      and the episode stops if close_2_goal was reported before this tick (the driver's
//                      real_close check precedes the close2goal update, main_sim_mpc.py:124-135)
// ------------------------------------------------------------------------------------------------
struct CLP {
    long long B;
    long long b0;     // global index of episode 0 of this launch (an episode group's offset: the kick's seed index)
    int S, f, s, i, variant, N;
    double ch_r, shb_r, bsh_r, tr;   // ALIP flow over rest_t: cosh, sinh / beta, beta sinh, rest_t / T
    double ch_d, shb_d, bsh_d, td;   // ... over dt = T / f_cyc
    double kick;
    unsigned long long seed;
    const double* goal;
    double* x;        // B x 5 plant state
    double* pst;      // B x 2 stance foot
    double* hdv;      // B x 4: nex_turn, hd_input_pr, hd_input_cos, -
    double* mhd;      // B x 3 mpc_hds_list
    double* plan;     // B x 5N mpc_state_tar
    int8_t* leg;      // B leg_ind
    uint8_t* flags;   // B: bit 0 active, bit 1 has a plan, bit 2 real_close
    double* xs;       // solve inputs
    double* u0;
    int8_t* sleg;
    const double* u;  // solve outputs
    const double* foot;
    const double* x_pred;
    const int32_t* status;
    const int32_t* iters;
    uint8_t* active;  // the solve's active mask
    double* foot_traj;      // B x S x 3
    double* x_traj;         // B x (S+1) x 5
    double* hd_traj;        // B x S x 2
    int32_t* status_traj;   // B x S x f
    int32_t* iters_traj;    // B x S x f
    int32_t* steps_to_goal; // B
    // task-space-controller command per tick (Logger.gen_nex_foot_input / gen_tsc_control), optional
    double* action_traj;    // B x S x f x 8
    double* vdes;           // B x 2 v_des_map (main_sim_mpc.py:54, 88, 112)
    double* pose0;          // B x 3 the initial pose: origin / heading of the Logger's robot-global frame
    double vdx, vdy0;       // alip_des_vel(0.6, leg_ind) = [vdx, -0.25 * 0.3 * leg_ind * vdy0]
};

// Logger.angle_A_minus_B (logger_mpc.py:169-175)
__host__ __device__ inline double ang_diff(double A, double B)
{
    double r = A - B;
    if (r < 0 && fabs(r) > M_PI)
        r += 2 * M_PI;
    else if (r > 0 && fabs(r) > M_PI)
        r -= 2 * M_PI;
    return r;
}
// Logger.tube_func (logger_mpc.py:283-300)
__host__ __device__ inline double tube_turn(double turning, double init)
{
    double tv = init;
    if (turning > 0)
        tv += (0.15 > turning ? 0.4 : 0.7) * turning;
    else if (turning < 0)
        tv += (-0.15 < turning ? 0.4 : 0.7) * turning;
    return ang_diff(tv, init);
}

// splitmix64 -> uniform [0, 1): the plant's velocity kick of (episode, step, tick, axis)
__host__ __device__ inline double cl_uniform(unsigned long long seed, long long b, int s, int i, int axis)
{
    unsigned long long z = seed + 0x9E3779B97F4A7C15ull *
                                      (((((unsigned long long)b * 1048576ull + (unsigned long long)s) * 1024ull +
                                         (unsigned long long)i) * 2ull + (unsigned long long)axis) + 1ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z = z ^ (z >> 31);
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

__global__ __launch_bounds__(256) void cl_project_kernel(CLP C)
{
    const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= C.B) return;
    const uint8_t fl = C.flags[b];
    C.active[b] = fl & 1;
    if (!(fl & 1)) return;
    double* x = C.x + 5 * b;
    double* hv = C.hdv + 4 * b;
    const double* mh = C.mhd + 3 * b;
    if (C.i == 0) {
        // set_stf_head (logger_mpc.py:270-280) with the plant heading
        const double cur = x[4];
        hv[2] = cur;
        hv[0] = tube_turn(hv[0], cur);
        double sum = hv[0];
        const double nc[3] = {cur, mh[0], mh[1]};
        for (int k = 0; k < 3; ++k) sum += ang_diff(mh[k], nc[k]);
        hv[1] = sum / 4.0;
        if (C.hd_traj) {
            C.hd_traj[((size_t)b * C.S + C.s) * 2] = hv[1];
            C.hd_traj[((size_t)b * C.S + C.s) * 2 + 1] = hv[2];
        }
    }
    // get_next_states(pos, vel, hd, [foot, hd_input_pr], rest_t)
    const double fx = C.pst[2 * b], fy = C.pst[2 * b + 1], hp = hv[1];
    double xn[5];
    xn[0] = C.ch_r * x[0] + C.shb_r * x[2] + (1.0 - C.ch_r) * fx;
    xn[1] = C.ch_r * x[1] + C.shb_r * x[3] + (1.0 - C.ch_r) * fy;
    xn[2] = C.bsh_r * x[0] + C.ch_r * x[2] - C.bsh_r * fx;
    xn[3] = C.bsh_r * x[1] + C.ch_r * x[3] - C.bsh_r * fy;
    xn[4] = x[4] + C.tr * hp;
    for (int c = 0; c < 5; ++c) C.xs[5 * b + c] = xn[c];
    const int n = 5 * C.N;
    double* g = C.u0 + (size_t)b * n;
    const double* pl = C.plan + (size_t)b * n;
    if (!(fl & 2)) {
        for (int k = 0; k < C.N; ++k)
            for (int c = 0; c < 5; ++c) g[5 * k + c] = xn[c];
    } else if (C.variant == ALIPMPC_VARIANT_SIG_STEP) {
        for (int k = 0; k < C.N; ++k) {
            const int src = k + 1 < C.N ? k + 1 : C.N - 1;
            for (int c = 0; c < 5; ++c) g[5 * k + c] = pl[5 * src + c];
        }
    } else {
        for (int i = 0; i < n; ++i) g[i] = pl[i];
    }
    C.sleg[b] = (int8_t)(-C.leg[b]);
}

// launch order of the next tick's solve (wave program): instances by the iteration count of their last solve,
// longest first (a counting sort; ties in any order), so the instances that will take longest start first and
// the launch does not wait on a late-starting long instance (tools/placement.py: cfg2 0.604 -> 0.417 ms with the
// long instances first).  One workgroup; inactive instances go last.
constexpr int CL_ORDER_THREADS = 1024;
__global__ __launch_bounds__(CL_ORDER_THREADS) void cl_order_kernel(const int32_t* iters, const uint8_t* active,
                                                                    long long B, int32_t* order)
{
    constexpr int NK = 64;
    __shared__ unsigned hist[NK];
    const int t = threadIdx.x;
    auto key = [&](long long b) {
        if (active && !active[b]) return NK - 1;
        const int it = iters[b];
        return NK - 2 - (it < 0 ? 0 : (it > NK - 2 ? NK - 2 : it));
    };
    if (t < NK) hist[t] = 0u;
    __syncthreads();
    for (long long b = t; b < B; b += CL_ORDER_THREADS) atomicAdd(&hist[key(b)], 1u);
    __syncthreads();
    if (t == 0) {
        unsigned acc = 0;
        for (int k = 0; k < NK; ++k) {
            const unsigned c = hist[k];
            hist[k] = acc;
            acc += c;
        }
    }
    __syncthreads();
    for (long long b = t; b < B; b += CL_ORDER_THREADS) order[atomicAdd(&hist[key(b)], 1u)] = (int32_t)b;
}

__global__ __launch_bounds__(256) void cl_update_kernel(CLP C)
{
    const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= C.B) return;
    uint8_t fl = C.flags[b];
    const size_t ti = ((size_t)b * C.S + C.s) * C.f + C.i;
    if (!(fl & 1)) {
        if (C.status_traj) C.status_traj[ti] = ALIPMPC_ROLLOUT_DONE;
        if (C.iters_traj) C.iters_traj[ti] = 0;
        if (C.action_traj)
            for (int c = 0; c < 8; ++c) C.action_traj[ti * 8 + c] = NAN;
        if (C.i == C.f - 1) {
            if (C.foot_traj)
                for (int c = 0; c < 3; ++c) C.foot_traj[((size_t)b * C.S + C.s) * 3 + c] = NAN;
            if (C.x_traj)
                for (int c = 0; c < 5; ++c) C.x_traj[((size_t)b * (C.S + 1) + C.s + 1) * 5 + c] = C.x[5 * b + c];
        }
        return;
    }
    const int n = 5 * C.N;
    if (C.status_traj) C.status_traj[ti] = C.status[b];
    if (C.iters_traj) C.iters_traj[ti] = C.iters[b];
    const double* ub = C.u + (size_t)b * n;
    const double* xp = C.x_pred + (size_t)b * n;
    for (int i = 0; i < n; ++i) C.plan[(size_t)b * n + i] = ub[i];
    fl |= 2;
    double* hv = C.hdv + 4 * b;
    hv[0] = C.foot[3 * b + 2];   // nex_turn = nex_contr[2]
    for (int k = 0; k < 3 && k < C.N; ++k) C.mhd[3 * b + k] = xp[5 * k + 4];
    // close_2_goal of this solve (modi |pos_1 - goal| <= 0.15, MPC_LIP_modi.py:108-115; sig_step any step
    // <= 0.35, MPC_LIP_sig_step.py:104-111)
    const double gx_ = C.goal[2 * b], gy_ = C.goal[2 * b + 1];
    bool close = false;
    const int kmax = C.variant == ALIPMPC_VARIANT_SIG_STEP ? C.N : 1;
    const double rad = C.variant == ALIPMPC_VARIANT_MODI ? 0.15 : 0.35;
    for (int k = 0; k < kmax; ++k) {
        const double dx = xp[5 * k] - gx_, dy = xp[5 * k + 1] - gy_;
        close = close || sqrt(dx * dx + dy * dy) <= rad;
    }
    double* x = C.x + 5 * b;
    const double fx = C.pst[2 * b], fy = C.pst[2 * b + 1];
    if (C.action_traj) {
        // gen_nex_foot_input (logger_mpc.py:318-360) + gen_tsc_control (:374-384): robot-global frame = the
        // map frame moved to the initial pose (pos/vel_map_glo_2_robo_glo, :134-150); the foot frame is the
        // stance foot rotated by the base heading
        const double* p0 = C.pose0 + 3 * b;
        double s0, c0;
        sincos(p0[2], &s0, &c0);
        auto rob = [&](double px, double py, double& rx, double& ry) {
            const double dx = px - p0[0], dy = py - p0[1];
            rx = c0 * dx + s0 * dy;
            ry = -s0 * dx + c0 * dy;
        };
        double nsx, nsy, csx, csy, npx, npy;
        rob(C.foot[3 * b], C.foot[3 * b + 1], nsx, nsy);       // nex_stf_rob (p_list[0])
        rob(fx, fy, csx, csy);                                  // pos_stf_rob_glo_frame
        rob(C.xs[5 * b], C.xs[5 * b + 1], npx, npy);            // nex_pos_rob (x_nex of this tick)
        const double vx = C.vdes[2 * b], vy = C.vdes[2 * b + 1];
        const double nvx = c0 * vx + s0 * vy, nvy = -s0 * vx + c0 * vy;   // nex_vel_rob
        double sb, cb;
        sincos(x[4] - p0[2], &sb, &cb);                         // M_T of hd_base_rob_glo_fram
        double* a = C.action_traj + ti * 8;
        a[0] = cb * (nsx - csx) + sb * (nsy - csy);
        a[1] = -sb * (nsx - csx) + cb * (nsy - csy);
        a[2] = 0.0;
        a[3] = hv[1] / C.f * (C.i + 4.5) + (hv[2] - p0[2]);    // hd_input_pr ramp + hd_input_cos (robot frame)
        a[4] = cb * (npx - csx) + sb * (npy - csy);
        a[5] = -sb * (npx - csx) + cb * (npy - csy);
        a[6] = cb * nvx + sb * nvy;
        a[7] = 0.0;
        (void)nvy;
    }
    // vel_des <- mpc_state_tar[0][2:4] after every solve, [1][2:4] at touchdown (main_sim_mpc.py:88, 112)
    if (C.vdes) {
        const int kv = (C.i == C.f - 1 && C.N > 1) ? 1 : 0;
        C.vdes[2 * b] = xp[5 * kv + 2];
        C.vdes[2 * b + 1] = xp[5 * kv + 3];
    }
    // the plant moves dt around the stance foot (+ the velocity kick)
    double xn[5];
    xn[0] = C.ch_d * x[0] + C.shb_d * x[2] + (1.0 - C.ch_d) * fx;
    xn[1] = C.ch_d * x[1] + C.shb_d * x[3] + (1.0 - C.ch_d) * fy;
    xn[2] = C.bsh_d * x[0] + C.ch_d * x[2] - C.bsh_d * fx;
    xn[3] = C.bsh_d * x[1] + C.ch_d * x[3] - C.bsh_d * fy;
    xn[4] = x[4] + C.td * hv[1];
    if (C.kick > 0) {
        xn[2] += C.kick * (2.0 * cl_uniform(C.seed, C.b0 + b, C.s, C.i, 0) - 1.0);
        xn[3] += C.kick * (2.0 * cl_uniform(C.seed, C.b0 + b, C.s, C.i, 1) - 1.0);
    }
    for (int c = 0; c < 5; ++c) x[c] = xn[c];
    if (C.i == C.f - 1) {
        // touchdown: the planned foothold becomes the stance foot, stance switch
        C.pst[2 * b] = C.foot[3 * b];
        C.pst[2 * b + 1] = C.foot[3 * b + 1];
        C.leg[b] = (int8_t)(-C.leg[b]);
        if (C.foot_traj)
            for (int c = 0; c < 3; ++c) C.foot_traj[((size_t)b * C.S + C.s) * 3 + c] = C.foot[3 * b + c];
        if (C.x_traj)
            for (int c = 0; c < 5; ++c) C.x_traj[((size_t)b * (C.S + 1) + C.s + 1) * 5 + c] = xn[c];
        if (fl & 4) {
            fl &= (uint8_t)~1u;
            if (C.steps_to_goal) C.steps_to_goal[b] = C.s + 1;
        }
    }
    if (close) fl |= 4;
    C.flags[b] = fl;
}

__global__ __launch_bounds__(256) void cl_init_kernel(CLP C)
{
    const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= C.B) return;
    C.flags[b] = 1;
    for (int k = 0; k < 4; ++k) C.hdv[4 * b + k] = 0.0;   // nex_turn = 0 (logger_mpc.py:90)
    // mpc_hds_list = [0, 0, 0] in the Logger's robot frame, whose origin is the initial pose (logger_mpc.py:27):
    // the initial heading in the map frame the plant and the MPC share here
    for (int k = 0; k < 3; ++k) C.mhd[3 * b + k] = C.x[5 * b + 4];
    if (C.steps_to_goal) C.steps_to_goal[b] = -1;
    if (C.x_traj)
        for (int c = 0; c < 5; ++c) C.x_traj[(size_t)b * (C.S + 1) * 5 + c] = C.x[5 * b + c];
    if (C.vdes) {   // vel_des = alip_des_vel(0.6, leg_ind) (main_sim_mpc.py:54)
        C.vdes[2 * b] = C.vdx;
        C.vdes[2 * b + 1] = 0.5 * (-0.5 * (double)C.leg[b] * 0.3) * C.vdy0;
        C.pose0[3 * b] = C.x[5 * b];
        C.pose0[3 * b + 1] = C.x[5 * b + 1];
        C.pose0[3 * b + 2] = C.x[5 * b + 4];
    }
}

// nominal gait (MPC_LIP_modi.py:181-194): vel_des = alip_des_vel(vx_max, leg_ind) unless a target velocity is
// given, foot = cal_foot_with_veldes(x, vel_des) = B_vel^-1 (vel_des - (A x)[2:4]) with B_vel = -beta sinh(beta T) I
struct NgP {
    long long B;
    double vdx, vdy0;     // sigma vx_max T / 2 and -0.25 step_gap beta sinh(beta T) / (cosh(beta T) + 1) per unit leg_ind
    double bsh, ch, ibv;  // beta sinh(beta T), cosh(beta T), 1 / (-beta sinh(beta T))
    const double* x;
    const int8_t* leg;
    const double* vin;
    double* vout;
    double* foot;
};
__global__ __launch_bounds__(256) void nominal_gait_kernel(NgP Q)
{
    const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= Q.B) return;
    const double* x = Q.x + 5 * b;
    double v0, v1;
    if (Q.vin) {
        v0 = Q.vin[2 * b];
        v1 = Q.vin[2 * b + 1];
    } else {
        v0 = Q.vdx;
        v1 = 0.5 * (-0.5 * (double)Q.leg[b] * 0.3) * Q.vdy0;
    }
    if (Q.vout) {
        Q.vout[2 * b] = v0;
        Q.vout[2 * b + 1] = v1;
    }
    const double ax = Q.bsh * x[0] + Q.ch * x[2], ay = Q.bsh * x[1] + Q.ch * x[3];
    Q.foot[2 * b] = Q.ibv * (v0 - ax);
    Q.foot[2 * b + 1] = Q.ibv * (v1 - ay);
}

// ------------------------------------------------------------------------------------------------
// dense CoM traces of a plan (the pos_det output of MPCCBF.gen_control_test, MPC_LIP_modi.py:117-122,
// 304-322): for step k, rows [x_k[0:2]; pos(t_i)], t_i = i * 0.01 (np.arange(0, dt + 0.01, 0.01)), of the
// continuous ALIP flow from x_k around the stance foot p_k:  pos(t) = ch x_k[0:2] + sh/beta x_k[2:4] +
// (1 - ch) p_k[0:2].  x_{k+1} = M_A x_k + M_B u_k and p_k = W (u_k - A x_k) as gen_control_test forms them.
// One thread per output row (coalesced 16-byte stores); HBM-bound: 40 B of plan in, rows x 16 B out.
// ------------------------------------------------------------------------------------------------
struct TrP {
    long long B;
    int N, rows;        // rows per step = 1 + samples
    double beta, step;  // sample spacing 0.01
    double A[25], W[15], MA[25], MB[25];
    const double* x0;   // B x 5
    const double* u;    // B x 5N
    double* trace;      // B x N x rows x 2
};

__global__ __launch_bounds__(256) void trace_kernel(TrP T)
{
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long per = (long long)T.N * T.rows;
    if (gid >= T.B * per) return;
    const long long b = gid / per;
    const int rem = (int)(gid - b * per), k = rem / T.rows, r = rem - k * T.rows;
    const double* ub = T.u + (size_t)b * 5 * T.N;
    double x[5];
    for (int i = 0; i < 5; ++i) x[i] = T.x0[(size_t)b * 5 + i];
    for (int j = 0; j < k; ++j) {   // x_{j+1} = M_A x_j + M_B u_j
        double y[5];
        for (int i = 0; i < 5; ++i) {
            double v = 0.0;
            for (int c = 0; c < 5; ++c) v += T.MA[i * 5 + c] * x[c];
            for (int c = 0; c < 5; ++c) v += T.MB[i * 5 + c] * ub[5 * j + c];
            y[i] = v;
        }
        for (int i = 0; i < 5; ++i) x[i] = y[i];
    }
    double px = x[0], py = x[1];
    if (r > 0) {
        double ax[5], p[2];
        for (int i = 0; i < 5; ++i) {
            double v = 0.0;
            for (int c = 0; c < 5; ++c) v += T.A[i * 5 + c] * x[c];
            ax[i] = ub[5 * k + i] - v;
        }
        for (int i = 0; i < 2; ++i) {
            double v = 0.0;
            for (int c = 0; c < 5; ++c) v += T.W[i * 5 + c] * ax[c];
            p[i] = v;
        }
        const double t = (r - 1) * T.step;
        const double ch = cosh(T.beta * t), sh = sinh(T.beta * t);
        px = ch * x[0] + sh / T.beta * x[2] + (1 - ch) * p[0];
        py = ch * x[1] + sh / T.beta * x[3] + (1 - ch) * p[1];
    }
    reinterpret_cast<double2*>(T.trace)[gid] = make_double2(px, py);
}
#endif  // ALIP_PART_HOST

// ------------------------------------------------------------------------------------------------
// kernel launchers.  The library may be built as one translation unit per horizon N (ALIP_PART = N:
// that horizon's kernels and launch_lip_N / launch_dd_N) plus ALIP_PART = 0 (host code, C ABI, rollout
// kernels), compiled in parallel and linked into one .so; without ALIP_PART everything is one TU.
// ------------------------------------------------------------------------------------------------
// dynamic-LDS opt-in, once per kernel and size (hipFuncSetAttribute is a host round trip: keep it out of the
// steady-state launch path)
static void set_smem(const void* f, size_t smem)
{
    static std::mutex mtx;
    static std::unordered_map<const void*, size_t> done[64];   // per device ordinal
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mtx);
    auto& d = done[dev & 63];
    auto it = d.find(f);
    if (it != d.end() && it->second >= smem) return;
    // (r5a: at N = 6 this call failed for a kernel variant that was not launched — its workgroup's LDS above the CU's
    // 160 KB — and the error it left was picked up by the launch's hipGetLastError, so every N = 6 solve reported
    // "invalid argument".  A failure is consumed here; launching a kernel whose LDS does not fit fails on its own.)
    if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem) != hipSuccess) {
        (void)hipGetLastError();
        return;
    }
    d[f] = smem;
}

// workgroups of kernel f resident on the whole device at once (occupancy x CUs), cached per (f, smem)
static unsigned resident_blocks(const void* f, size_t smem, int threads = WAVE * WAVES_PER_BLOCK)
{
    static std::mutex mtx;
    static std::map<std::pair<const void*, size_t>, unsigned> cache[64];
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mtx);
    auto& c = cache[dev & 63];
    auto it = c.find({f, smem});
    if (it != c.end()) return it->second;
    int per_cu = 0, cus = 0;
    unsigned r = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, threads, smem) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && per_cu > 0 && cus > 0)
        r = (unsigned)per_cu * (unsigned)cus;
    c[{f, smem}] = r;
    return r;
}

// the team-capable build's workgroup LDS: smem (KP, G and WAVES_PER_BLOCK workspaces) with TEAM_WAVES workspaces
template <int N, class R>
size_t team_smem(size_t smem)
{
    const size_t fixed = sizeof(double) * (size_t)KP_DOUBLES + sizeof(R) * (size_t)Dim<N>::NG * Dim<N>::NCP;
    return fixed + (smem - fixed) / WAVES_PER_BLOCK * TEAM_WAVES;
}

template <int N, class R>
void launch_solve(const KP& P0, size_t smem, hipStream_t st, unsigned* res_out)
{
    const unsigned need = (unsigned)((P0.B + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK);
    // a split launch with team records (team-capable build, TEAM_WAVES-wave workgroups); phase 2: P0.team team
    // workgroups ahead of the one-wave-per-instance ones
    const unsigned need_t = (P0.resume ? (unsigned)P0.team : 0u) + (unsigned)((P0.B + TEAM_WAVES - 1) / TEAM_WAVES);
    const size_t smem_t = team_smem<N, R>(smem);
    // KSM = 4-row steps of the J layout, the smallest compiled size covering mo4 rows
    auto go = [&](auto kq, auto k1, auto kt) {
        set_smem((const void*)kq, smem);
        set_smem((const void*)k1, smem);
        // (the team-capable build runs only where its workgroup fits the LDS: alipmpc_create clears the trial cuts
        // otherwise)
        if (smem_t <= 160 * 1024) set_smem((const void*)kt, smem_t);
        const unsigned res = resident_blocks((const void*)kq, smem);
        if (res_out) {   // query only (alipmpc_solve_slots)
            *res_out = res;
            return;
        }
        if (res > 0 && (need > res || P0.bcount) && !P0.resume)   // the persistent work queue over the resident workgroups
            hipLaunchKernelGGL(kq, dim3(res), dim3(WAVE * WAVES_PER_BLOCK), smem, st, P0);
        else if (P0.team > 0)        // a split launch with team records: both phases on the team-capable build
            hipLaunchKernelGGL(kt, dim3(need_t > 0 ? need_t : 1u), dim3(WAVE * TEAM_WAVES), smem_t, st, P0);
        else                         // every instance has a resident wave: one instance per wave
            hipLaunchKernelGGL(k1, dim3(need > 0 ? need : 1u), dim3(WAVE * WAVES_PER_BLOCK), smem, st, P0);
    };
    // the team-capable build exists in fp64 only: in fp32 its different code rounded differently from the plain build's
    // (fp32 contraction / packing decisions depend on the surrounding code), so fp32 splits never make team records
    // cfg.restoration = IPOPT: the restoration-capable builds, except for phase 1 of a split launch (records: a pending
    // restoration is cut to phase 2); the query of the resident slots uses the lean work-queue build either way
    // (fp32 has the lean build only: a failed search hands the instance to the fp64 wave program)
    const bool rs = P0.resto_ipopt && !(P0.ckpt && !P0.resume) && !res_out;
#define ALIP_GO(K)                                                                                              \
    do {                                                                                                        \
        if constexpr (sizeof(R) == 8) {                                                                         \
            if (rs)                                                                                             \
                go(solve_kernel<N, K, R, false, false, true>, solve_kernel<N, K, R, true, false, true>,         \
                   solve_kernel<N, K, R, true, true, true>);                                                    \
            else                                                                                                \
                go(solve_kernel<N, K, R, false>, solve_kernel<N, K, R, true>, solve_kernel<N, K, R, true, true>); \
        } else {                                                                                                \
            go(solve_kernel<N, K, R, false>, solve_kernel<N, K, R, true>, solve_kernel<N, K, R, true, false>);  \
        }                                                                                                       \
    } while (0)
#ifdef ALIP_DEV_ONLY_KSM   // dev builds for register reports (tools/regs.py): one row-step count only
    ALIP_GO(ALIP_DEV_ONLY_KSM);
#else
    if (P0.mo4 <= 16)   // (r5: sig_step / modi with no obstacle slots at N <= 3, cfg1: 0.1255 -> 0.1195 ms)
        ALIP_GO(4);
    else if (P0.mo4 <= 32)
        ALIP_GO(8);
    else if (P0.mo4 <= 40)
        ALIP_GO(10);
    else if (P0.mo4 <= 48)
        ALIP_GO(12);
    else if (P0.mo4 <= 64)
        ALIP_GO(16);
    else if (P0.mo4 <= 96)
        ALIP_GO(24);
    else if (P0.mo4 <= 128)
        ALIP_GO(32);
    else
        ALIP_GO(48);
#endif
#undef ALIP_GO
}

// solve kernels run in the handle's precision (cfg.precision); the eval hook is always fp64
template <int N>
hipError_t launch_t(bool solve, bool f32, const KP& P, size_t smem, hipStream_t st, unsigned* res_out)
{
    if (solve && f32) {
#ifndef ALIP_DEV_ONLY_KSM
        launch_solve<N, float>(P, smem, st, res_out);
#endif
    } else if (solve) {
        launch_solve<N, double>(P, smem, st, res_out);
    } else {
        // grid-stride eval kernel (16 instances per workgroup): at most the resident workgroups
        set_smem((const void*)eval_kernel<N>, smem);
        const unsigned need = (unsigned)((P.B + GROUPS_PER_BLOCK - 1) / GROUPS_PER_BLOCK);
        const unsigned res = resident_blocks((const void*)eval_kernel<N>, smem);
        const unsigned egrid = res > 0 && res < need ? res : (need > 0 ? need : 1u);
        hipLaunchKernelGGL(eval_kernel<N>, dim3(egrid), dim3(WAVE * WAVES_PER_BLOCK), smem, st, P);
    }
    return hipGetLastError();
}

template <int N>
hipError_t launch_dd(bool solve, const KP& P, size_t smem, hipStream_t st)
{
    const unsigned grid = (unsigned)((P.B + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK);
    auto go = [&](auto kern) {
        set_smem((const void*)kern, smem);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(WAVE * WAVES_PER_BLOCK), smem, st, P);
    };
    if (!solve)
        go(dd_eval_kernel<N>);
    else if (P.mo4 <= WAVE)
        go(dd_solve_kernel<N, 1>);
    else if (P.mo4 <= 2 * WAVE)
        go(dd_solve_kernel<N, 2>);
    else
        go(dd_solve_kernel<N, 3>);
    return hipGetLastError();
}

#define ALIP_LAUNCHERS(k)                                                                              \
    hipError_t launch_lip_##k(bool solve, bool f32, const KP& P, size_t smem, hipStream_t st,          \
                              unsigned* res_out)                                                       \
    {                                                                                                  \
        return launch_t<k>(solve, f32, P, smem, st, res_out);                                          \
    }                                                                                                  \
    hipError_t launch_dd_##k(bool solve, const KP& P, size_t smem, hipStream_t st)                     \
    {                                                                                                  \
        return launch_dd<k>(solve, P, smem, st);                                                       \
    }
#define ALIP_LAUNCH_DECL(k)                                                                            \
    hipError_t launch_lip_##k(bool solve, bool f32, const KP& P, size_t smem, hipStream_t st,          \
                              unsigned* res_out = nullptr);                                            \
    hipError_t launch_dd_##k(bool solve, const KP& P, size_t smem, hipStream_t st);
ALIP_LAUNCH_DECL(1) ALIP_LAUNCH_DECL(2) ALIP_LAUNCH_DECL(3) ALIP_LAUNCH_DECL(4) ALIP_LAUNCH_DECL(5) ALIP_LAUNCH_DECL(6)
#if ALIP_PART_N(1)
ALIP_LAUNCHERS(1)
#endif
#if ALIP_PART_N(2)
ALIP_LAUNCHERS(2)
#endif
#if ALIP_PART_N(3)
ALIP_LAUNCHERS(3)
#endif
#if ALIP_PART_N(4)
ALIP_LAUNCHERS(4)
#endif
#if ALIP_PART_N(5)
ALIP_LAUNCHERS(5)
#endif
#if ALIP_PART_N(6)
ALIP_LAUNCHERS(6)
#endif

// lane solver (lane_solve.inc): N = 3, circles only, NC = compiled circle slots (>= cfg.nc_max).  A persistent
// grid of at most the resident one-wave workgroups; each lane takes instances from the launch's work queue.
template <int N, int NC, bool MODI, class R>
void launch_lane_t(const KP& P, hipStream_t st, unsigned* res_out)
{
    auto kern = lane_kernel<N, NC, MODI, R>;
    const unsigned res = resident_blocks((const void*)kern, 0, WAVE);
    if (res_out) {
        *res_out = res;
        return;
    }
    const unsigned need = (unsigned)((P.B + WAVE - 1) / WAVE);
    // small batches are spread over every resident wave (the kernel's first fetch takes ceil(B / grid))
    const unsigned grid = res > 0 ? res : (need > 0 ? need : 1u);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(WAVE), 0, st, P);
}
template <class R>
hipError_t launch_lane_r(int nct, bool modi, const KP& P, hipStream_t st, unsigned* res_out)
{
    if (modi) {
        if (nct == 0) launch_lane_t<3, 0, true, R>(P, st, res_out);
        else if (nct == 5) launch_lane_t<3, 5, true, R>(P, st, res_out);
        else if (nct == 6) launch_lane_t<3, 6, true, R>(P, st, res_out);
        else return hipErrorInvalidValue;
    } else {
        if (nct == 0) launch_lane_t<3, 0, false, R>(P, st, res_out);
        else if (nct == 5) launch_lane_t<3, 5, false, R>(P, st, res_out);
        else if (nct == 6) launch_lane_t<3, 6, false, R>(P, st, res_out);
        else return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
hipError_t launch_lane_f64(int nct, bool modi, const KP& P, hipStream_t st, unsigned* res_out);
hipError_t launch_lane_f32(int nct, bool modi, const KP& P, hipStream_t st, unsigned* res_out);
#if !defined(ALIP_PART) || ALIP_PART == 7
hipError_t launch_lane_f64(int nct, bool modi, const KP& P, hipStream_t st, unsigned* res_out)
{
    return launch_lane_r<double>(nct, modi, P, st, res_out);
}
#endif
#if !defined(ALIP_PART) || ALIP_PART == 8
hipError_t launch_lane_f32(int nct, bool modi, const KP& P, hipStream_t st, unsigned* res_out)
{
    return launch_lane_r<float>(nct, modi, P, st, res_out);
}
#endif

// sweep kernel (eval hook, N = 3, circles only): CH-instance chunks per wave, WPG waves per workgroup, a grid-stride
// over the chunks on at most the resident workgroups
hipError_t launch_sweep(int nc, bool fen, const KP& P, hipStream_t st);
#if ALIP_PART_N(3)
template <int NC, bool FEN, int CH, int WPG>
void launch_sweep_t(const KP& P, hipStream_t st)
{
    using L = SweepL<NC, FEN>;
    auto kern = sweep_kernel<NC, FEN, CH, WPG>;
    const size_t smem = sizeof(double) * ((size_t)L::GL + (size_t)WPG * (CH / 2) * L::SLOTD);
    set_smem((const void*)kern, smem);
    const unsigned res = resident_blocks((const void*)kern, smem, WAVE * WPG);
    const long long per = (long long)CH * WPG;
    const unsigned need = (unsigned)((P.B + per - 1) / per);
    const unsigned grid = res > 0 && res < need ? res : (need > 0 ? need : 1u);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(WAVE * WPG), smem, st, P);
}
template <int NC, bool FEN>
void launch_sweep_s(const KP& P, hipStream_t st)
{
    // instances per wave x waves per workgroup (LDS: the G/E copy per workgroup + CH/2 coefficient slots per
    // wave); ALIPMPC_SWEEP_SHAPE (dev A/B) picks another shape
    const char* se = getenv("ALIPMPC_SWEEP_SHAPE");
    const int shape = se ? atoi(se) : SWEEP_SHAPE_DEFAULT;
    // measured (profiles/r2/sweep/shapes.txt, B = 65,536): 64 x 1 0.0837 ms (one wave per SIMD: the LDS of a
    // 64-instance chunk), 32 x 2 0.0759 ms (two per SIMD, 2048 waves), 16 x 4 0.106 ms (232 VGPRs cap the SIMD at
    // two waves, and each wave repeats the set-up for a quarter of the instances)
    if (shape == 641)
        launch_sweep_t<NC, FEN, 64, 1>(P, st);
    else
        launch_sweep_t<NC, FEN, 32, 2>(P, st);
}
hipError_t launch_sweep(int nc, bool fen, const KP& P, hipStream_t st)
{
#define SWCASE(K)                                              \
    case K:                                                    \
        fen ? launch_sweep_s<K, true>(P, st) : launch_sweep_s<K, false>(P, st); \
        break;
    switch (nc) {
        SWCASE(0) SWCASE(1) SWCASE(2) SWCASE(3) SWCASE(4) SWCASE(5) SWCASE(6)
    default:
        return hipErrorInvalidValue;
    }
#undef SWCASE
    return hipGetLastError();
}
#endif

}  // namespace alip

#if ALIP_PART_HOST
// ================================================================================================
// host side: constants, handle, C ABI
// ================================================================================================
namespace {

using namespace alip;

struct Handle {
    alipmpc_cfg cfg;
    int device = 0;
    int N = 3, n = 9, NG = 32, NCP = 16, NCPU = 16, rps = 0, m_max = 0, mr4 = 0;
    int rps_s = 0, m_s = 0, mr4_s = 0, mo4 = 0;   // solve-kernel row layout (f_en split, objective rows)
    double* dGp = nullptr;
    double* dEp = nullptr;
    double* dGu = nullptr;
    double* dEu = nullptr;
    // lane solver (lane_solve.inc): constants and the compiled circle-slot count it runs with (-1: the
    // per-wave solve_kernel serves this configuration)
    double* dlk = nullptr;
    float* dlkf = nullptr;
    int lane_nct = -1;
    // eval hook: the circle-slot count sweep_kernel runs with (-1: eval_kernel serves this configuration)
    int sweep_nc = -1;
    // work-queue counter pairs of persistent solve launches (a ring: launches in flight on different
    // streams use different pairs; each pair is reset by the last wave of the launch that used it), followed by
    // MAXG pairs owned by the closed loop's episode groups (one per group)
    static constexpr unsigned NQ = 64;
    uint32_t* dq = nullptr;
    mutable std::atomic<unsigned> qi{0};
    // staging for host-pointer calls
    void* stage = nullptr;
    size_t stage_bytes = 0;
    // rollout working set (evolving state, warm starts, per-step solve outputs)
    void* rstage = nullptr;
    size_t rstage_bytes = 0;
    hipStream_t own = nullptr;
    // closed loop: episode groups on streams of their own (ALIPMPC_CL_GROUPS), fork / join events
    static constexpr int MAXG = 8;
    hipStream_t gst[MAXG] = {};
    hipEvent_t gev[MAXG + 1] = {};
    // split launch of the wave program (ALIPMPC_SPLIT_IT): the phase-1 iteration cap (0 = off) and, per stream, the
    // record buffer (launches on one stream run in order, so they may share it; other streams get their own)
    int split_it = 0;
    int split_tr = 0;   // phase-1 trial cut: an instance at this many line-search trials resumes as a team (0 = off)
    int cl_split_it = 0, cl_split_tr = 0;   // the closed loop's per-tick solves (ALIPMPC_CL_SPLIT_IT / _TR)
    // Record buffers are sized ONCE for the resident slots (the largest batch that splits) and never reallocated or
    // freed before alipmpc_destroy, so a graph captured on a stream keeps a valid pointer whatever batch sizes run on
    // that stream later.  At most SPLIT_STREAMS of them: a further stream runs the one-phase form.
    static constexpr size_t SPLIT_STREAMS = 8;
    struct SplitBuf {
        void* p = nullptr;
        size_t bytes = 0;
    };
    std::map<hipStream_t, SplitBuf> split;
    std::mutex split_mtx;
    // lane program with cfg.restoration = IPOPT: per stream, the list of instances handed to the wave program (count +
    // indices; grown to the largest batch seen, never freed before alipmpc_destroy)
    std::map<hipStream_t, SplitBuf> redo;
    // launch timing: a ring of event pairs, so a re-record never targets an event still pending on the
    // stream (that serialises the host with the previous launch)
    static constexpr int NEV = 16;
    hipEvent_t ev[NEV][2] = {};
    int evi = 0, evlast = -1;
    bool timed = false;
    std::string err;
};

int fail(Handle* h, int code, const std::string& msg)
{
    if (h) h->err = msg;
    return code;
}

#define HIPCHK(h, x)                                                                            \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) return fail(h, ALIPMPC_EHIP, std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)

void mm(const double* a, const double* b, double* c, int n1, int n2, int n3)
{
    for (int i = 0; i < n1; ++i)
        for (int j = 0; j < n3; ++j) {
            double s = 0;
            for (int k = 0; k < n2; ++k) s += a[i * n2 + k] * b[k * n3 + j];
            c[i * n3 + j] = s;
        }
}

// generator tables.  Row 8k+c (c<5): state x_k[c]; row 8k+5+c (c<3): foothold p_k[c]; V = E x0 + G z.
//  u-parametrisation (the reference's decision, eval + warm start): x_{k+1} = M_A x_k + M_B u_k,
//    p_k = W(u_k - A x_k)                                           (MPC_LIP_modi.py:64-87, 630-634)
//  foothold parametrisation (the solve): x_{k+1} = A x_k + B p_k   (W B = I, so the two describe the same
//    NLP; u enters it only through W u_k, which leaves a 2N-dim null space in u that p removes)
void build_tables(const alipmpc_cfg& cfg, int NCPP, int NCPU, std::vector<double>& Gp, std::vector<double>& Ep,
                  std::vector<double>& Gu, std::vector<double>& Eu)
{
    const int N = cfg.N, n = 5 * N, np_ = 3 * N, NG = 8 * (N + 1);
    const double b = std::sqrt(cfg.g / cfg.H), T = cfg.dt;
    const double ch = std::cosh(b * T), sh = std::sinh(b * T);
    double A[25] = {ch, 0, sh / b, 0, 0, 0, ch, 0, sh / b, 0, sh * b, 0, ch, 0, 0, 0, sh * b, 0, ch, 0, 0, 0, 0, 0, 1};
    double Bm[15] = {1 - ch, 0, 0, 0, 1 - ch, 0, -sh * b, 0, 0, 0, -sh * b, 0, 0, 0, 1};
    const double a_ = 5.0, b_ = 1.0;
    const double Dd = a_ * (ch - 1) * (ch - 1) + b_ * (sh * b) * (sh * b);
    const double Ch = -a_ * (ch - 1) / Dd, Sh = -b_ * sh * b / Dd;
    double W[15] = {Ch, 0, Sh, 0, 0, 0, Ch, 0, Sh, 0, 0, 0, 0, 0, 1};
    double MB[25], BWA[25], MA[25], WA[15];
    mm(Bm, W, MB, 5, 3, 5);
    mm(MB, A, BWA, 5, 5, 5);
    for (int i = 0; i < 25; ++i) MA[i] = A[i] - BWA[i];
    mm(W, A, WA, 3, 5, 5);
    // ---- u tables
    std::vector<double> Phi((N + 1) * 5 * n, 0.0), Pk((N + 1) * 25, 0.0);
    for (int i = 0; i < 5; ++i) Pk[i * 5 + i] = 1.0;
    for (int k = 1; k <= N; ++k) {
        mm(MA, &Phi[(k - 1) * 5 * n], &Phi[k * 5 * n], 5, 5, n);
        for (int i = 0; i < 5; ++i)
            for (int j = 0; j < 5; ++j) Phi[k * 5 * n + i * n + 5 * (k - 1) + j] += MB[i * 5 + j];
        mm(MA, &Pk[(k - 1) * 25], &Pk[k * 25], 5, 5, 5);
    }
    Gu.assign((size_t)NG * NCPU, 0.0);
    Eu.assign((size_t)NG * 5, 0.0);
    for (int k = 0; k <= N; ++k) {
        for (int c = 0; c < 5; ++c) {
            for (int j = 0; j < n; ++j) Gu[(8 * k + c) * NCPU + j] = Phi[k * 5 * n + c * n + j];
            for (int j = 0; j < 5; ++j) Eu[(8 * k + c) * 5 + j] = Pk[k * 25 + c * 5 + j];
        }
        if (k < N) {
            std::vector<double> WAPhi(3 * n), WAPk(15);
            mm(WA, &Phi[k * 5 * n], WAPhi.data(), 3, 5, n);
            mm(WA, &Pk[k * 25], WAPk.data(), 3, 5, 5);
            for (int c = 0; c < 3; ++c) {
                for (int j = 0; j < n; ++j) Gu[(8 * k + 5 + c) * NCPU + j] = -WAPhi[c * n + j];
                for (int j = 0; j < 5; ++j) Gu[(8 * k + 5 + c) * NCPU + 5 * k + j] += W[c * 5 + j];
                for (int j = 0; j < 5; ++j) Eu[(8 * k + 5 + c) * 5 + j] = -WAPk[c * 5 + j];
            }
        }
    }
    // ---- foothold tables: x_k = A^k x0 + sum_{j<k} A^{k-1-j} B p_j
    std::vector<double> Ak((N + 1) * 25, 0.0);
    for (int i = 0; i < 5; ++i) Ak[i * 5 + i] = 1.0;
    for (int k = 1; k <= N; ++k) mm(A, &Ak[(k - 1) * 25], &Ak[k * 25], 5, 5, 5);
    Gp.assign((size_t)NG * NCPP, 0.0);
    Ep.assign((size_t)NG * 5, 0.0);
    for (int k = 0; k <= N; ++k) {
        for (int c = 0; c < 5; ++c) {
            for (int j = 0; j < 5; ++j) Ep[(8 * k + c) * 5 + j] = Ak[k * 25 + c * 5 + j];
            for (int jj = 0; jj < k; ++jj) {
                double AB[15];
                mm(&Ak[(k - 1 - jj) * 25], Bm, AB, 5, 5, 3);
                for (int c2 = 0; c2 < 3; ++c2) Gp[(8 * k + c) * NCPP + 3 * jj + c2] = AB[c * 3 + c2];
            }
        }
        if (k < N)
            for (int c = 0; c < 3; ++c) Gp[(8 * k + 5 + c) * NCPP + 3 * k + c] = 1.0;
    }
    (void)np_;
}

// lane-solver constants (lane::LK_* slots): the ALIP step map per axis, W, the foothold sensitivities
// d px_k / d fx_j = (Abar^(k-1-j) bbar)[0] and d vx_k / d fx_j = (...)[1], the relaxed (IPOPT
// bound_relax_factor 1e-8, as the oracle) and original bounds, weights and tolerances
void lane_constants(const alipmpc_cfg& cfg, double* lk)
{
    using namespace alip::lane;
    static_assert(LK_COUNT <= LK_BUF, "lane constants fit their buffer");
    for (int i = 0; i < LK_BUF; ++i) lk[i] = 0.0;
    const double b = std::sqrt(cfg.g / cfg.H), T = cfg.dt;
    const double ch = std::cosh(b * T), sh = std::sinh(b * T);
    lk[LK_CH] = ch;
    lk[LK_SHB] = sh / b;
    lk[LK_BSH] = sh * b;
    lk[LK_OMC] = 1.0 - ch;
    const double a_ = 5.0, b_ = 1.0;
    const double Dd = a_ * (ch - 1) * (ch - 1) + b_ * (sh * b) * (sh * b);
    lk[LK_WCH] = -a_ * (ch - 1) / Dd;
    lk[LK_WSH] = -b_ * sh * b / Dd;
    double v0 = 1.0 - ch, v1 = -sh * b;
    for (int m = 0; m < 6; ++m) {
        lk[LK_SP + m] = v0;
        lk[LK_SV + m] = v1;
        const double w0 = ch * v0 + (sh / b) * v1, w1 = sh * b * v0 + ch * v1;
        v0 = w0;
        v1 = w1;
    }
    auto rl = [](double x) { return x - 1e-8 * std::fmax(1.0, std::fabs(x)); };
    auto ru = [](double x) { return x + 1e-8 * std::fmax(1.0, std::fabs(x)); };
    lk[LK_VXL] = rl(cfg.bvx_lo);
    lk[LK_VXU] = ru(cfg.bvx_hi);
    lk[LK_VYLP] = rl(cfg.bvy_lo);
    lk[LK_VYUP] = ru(cfg.bvy_hi);
    lk[LK_VYLN] = rl(-cfg.bvy_hi);
    lk[LK_VYUN] = ru(-cfg.bvy_lo);
    lk[LK_CIRL] = rl(0.0);
    lk[LK_LEGL] = rl(0.0);
    lk[LK_LEGU] = ru(cfg.leg2_max);
    lk[LK_DTL] = rl(-cfg.dtheta_max);
    lk[LK_DTU] = ru(cfg.dtheta_max);
    lk[LK_OVXL] = cfg.bvx_lo;
    lk[LK_OVXU] = cfg.bvx_hi;
    lk[LK_OVYLP] = cfg.bvy_lo;
    lk[LK_OVYUP] = cfg.bvy_hi;
    lk[LK_OVYLN] = -cfg.bvy_hi;
    lk[LK_OVYUN] = -cfg.bvy_lo;
    lk[LK_OLEGU] = cfg.leg2_max;
    lk[LK_ODT] = cfg.dtheta_max;
    lk[LK_Q] = cfg.q;
    lk[LK_P] = cfg.p;
    lk[LK_R] = cfg.r;
    lk[LK_GM1] = cfg.gamma - 1.0;
    lk[LK_S] = cfg.s;
    lk[LK_TOL] = cfg.tol;
    lk[LK_ACC] = cfg.acceptable_tol;
    lk[LK_MU0] = cfg.mu_init;
    lk[LK_DET2] = cfg.detect_r2;
    // d px_{k+1+m} / d u_k[px], [vx] of the reference's u (per axis: (MA^m MB)[0][0], [0][1], MA = (I - B W) A, MB = B W),
    // for IPOPT's objective scaling at the starting point (lane_solve.inc)
    {
        const double Ax[2][2] = {{ch, sh / b}, {sh * b, ch}}, Bx[2] = {1.0 - ch, -sh * b};
        const double Wx[2] = {lk[LK_WCH], lk[LK_WSH]};
        double MA[2][2], MB[2][2], Mm[2][2] = {{1, 0}, {0, 1}};   // Mm = MA^m
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 2; ++j) {
                MB[i][j] = Bx[i] * Wx[j];
                MA[i][j] = Ax[i][j] - Bx[i] * (Wx[0] * Ax[0][j] + Wx[1] * Ax[1][j]);
            }
        for (int m = 0; m < 6; ++m) {
            lk[LK_SU0 + m] = Mm[0][0] * MB[0][0] + Mm[0][1] * MB[1][0];
            lk[LK_SU1 + m] = Mm[0][0] * MB[0][1] + Mm[0][1] * MB[1][1];
            double T[2][2];
            for (int i = 0; i < 2; ++i)
                for (int j = 0; j < 2; ++j) T[i][j] = Mm[i][0] * MA[0][j] + Mm[i][1] * MA[1][j];
            for (int i = 0; i < 2; ++i)
                for (int j = 0; j < 2; ++j) Mm[i][j] = T[i][j];
        }
    }
}

// the compiled lane-solver instance (circle slots) serving cfg, or -1 when none does: N = 3 with circles
// only (<= 6 slots), modi / sig_step (BASELINE cfg1/2/4/5 shapes)
int lane_slots_for(const alipmpc_cfg& c)
{
    if (c.variant == ALIPMPC_VARIANT_DD || c.N != 3 || c.ne_max != 0 || c.nc_max > 6) return -1;
    return c.nc_max == 0 ? 0 : c.nc_max <= 5 ? 5 : 6;
}

size_t smem_bytes(const Handle* h, bool solve, int force_f64 = 0)
{
    if (h->cfg.variant == ALIPMPC_VARIANT_DD) {
        int wsd = 0;
        switch (h->N) {
#define DDCASE(NN) \
    case NN: wsd = ddw_doubles<NN>(h->cfg.nc_max + h->cfg.ne_max, h->mo4); break;
            DDCASE(1) DDCASE(2) DDCASE(3) DDCASE(4) DDCASE(5) DDCASE(6)
#undef DDCASE
        }
        (void)solve;
        return sizeof(double) * ((size_t)KP_DOUBLES + (size_t)WAVES_PER_BLOCK * wsd);
    }
    const bool f32 = solve && h->cfg.precision == ALIPMPC_PREC_FP32 && !force_f64;
    int wsd = 0;
    switch (h->N) {
#define WSCASE(NN)                                                                                     \
    case NN:                                                                                           \
        wsd = solve ? (f32 ? wss_elems<NN, float>(h->cfg.nc_max, h->cfg.ne_max, h->mr4_s, h->mo4)      \
                           : wss_elems<NN, double>(h->cfg.nc_max, h->cfg.ne_max, h->mr4_s, h->mo4)) \
                    : gws_doubles<NN>(h->cfg.nc_max, h->cfg.ne_max, h->mr4);                           \
        break;
        WSCASE(1) WSCASE(2) WSCASE(3) WSCASE(4) WSCASE(5) WSCASE(6)
#undef WSCASE
    }
    const int e = solve ? 0 : h->NG * 5 + ((h->NG * 5) & 1);   // (solve_kernel: E from global memory)
    const int ncp = solve ? h->NCP : h->NCPU;
    // KP in fp64 units, then G, E and the per-wave workspaces in the kernel's arithmetic type
    const size_t per_block = solve ? (size_t)WAVES_PER_BLOCK : (size_t)GROUPS_PER_BLOCK;   // workspaces
    return sizeof(double) * (size_t)KP_DOUBLES +
           (f32 ? sizeof(float) : sizeof(double)) * ((size_t)h->NG * ncp + e + per_block * wsd);
}

KP make_kp(const Handle* h, long long B, bool solve)
{
    const alipmpc_cfg& c = h->cfg;
    KP P;
    std::memset(&P, 0, sizeof(P));
    P.nc_max = c.nc_max;
    P.ne_max = c.ne_max;
    P.rps = solve ? h->rps_s : h->rps;
    P.m_max = solve ? h->m_s : h->m_max;
    P.mr4 = solve ? h->mr4_s : h->mr4;
    P.mo4 = h->mo4;
    P.modi = c.variant == ALIPMPC_VARIANT_MODI;
    P.max_iter = c.max_iter;
    P.select_obs = c.select_obs;
    P.detour = c.detour;
    P.goal_abort = c.goal_singular == ALIPMPC_GOAL_SINGULAR_ABORT;
    P.resto_ipopt = c.restoration == ALIPMPC_RESTORATION_IPOPT && c.variant != ALIPMPC_VARIANT_DD;
    P.tol = c.tol;
    P.acc_tol = c.acceptable_tol;
    P.q = c.q;
    P.p = c.p;
    P.r = c.r;
    P.gm1 = c.gamma - 1.0;
    P.s = c.s;
    P.detect_r2 = c.detect_r2;
    P.leg2 = c.leg2_max;
    P.bvx_lo = c.bvx_lo;
    P.bvx_hi = c.bvx_hi;
    P.bvy_lo = c.bvy_lo;
    P.bvy_hi = c.bvy_hi;
    P.dth = c.dtheta_max;
    P.mu_init = c.mu_init;
    P.dt = c.dt;
    P.dd_t = c.dd_t;
    P.G = solve ? h->dGp : h->dGu;
    P.E = solve ? h->dEp : h->dEu;
    P.Gu = h->dGu;
    P.Eu = h->dEu;
    P.B = B;
    P.lkd = h->dlk;
    P.lkfd = h->dlkf;
    if (solve && c.variant != ALIPMPC_VARIANT_DD) P.queue = h->dq + 2 * (h->qi.fetch_add(1u) % Handle::NQ);
    return P;
}

// J-layout steps (4 rows each) of the compiled solve kernels; mo4 is rounded up to 4 * ksm_of(rows)
int ksm_of(int rows)
{
    static const int K[] = {4, 8, 10, 12, 16, 24, 32, 48};
    for (int k : K)
        if (rows <= 4 * k) return k;
    return 1 << 20;
}

// cfg.restoration = IPOPT, fp32 programs and the lane program: the stream's hand-off list ([0] = count, then the
// instances), allocated outside a capture (a capture needs an uncaptured solve of that size on the stream first)
static hipError_t redo_list(const Handle* h, hipStream_t st, long long B, uint32_t** out)
{
    Handle* hm = const_cast<Handle*>(h);
    std::lock_guard<std::mutex> lk(hm->split_mtx);
    Handle::SplitBuf& rb = hm->redo[st];
    const size_t need = sizeof(uint32_t) * (size_t)(B + 1);
    if (rb.bytes < need) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return hipErrorNotSupported;
        if (rb.p) {
            (void)hipStreamSynchronize(st);
            (void)hipFree(rb.p);
            rb.p = nullptr;
            rb.bytes = 0;
        }
        if (hipError_t e = hipMalloc(&rb.p, need)) return e;
        rb.bytes = need;
    }
    *out = (uint32_t*)rb.p;
    return hipSuccess;
}

// the listed instances, solved from their start by the fp64 wave program's restoration-capable work queue (slot k
// solves redo[1 + k], k < redo[0]) on the same stream
static hipError_t launch_handoff(const Handle* h, const KP& P, const uint32_t* redo, hipStream_t st)
{
    KP Q = P;
    Q.redo = nullptr;
    Q.order = reinterpret_cast<const int32_t*>(redo + 1);
    Q.bcount = redo;
    Q.ckpt = nullptr;
    Q.cont = nullptr;
    Q.resume = 0;
    Q.team = 0;
    Q.ckpt_it = 0;
    Q.ckpt_tr = 0;
    const size_t sm = smem_bytes(h, true, 1);
    switch (h->N) {
    case 1: return launch_lip_1(true, false, Q, sm, st, nullptr);
    case 2: return launch_lip_2(true, false, Q, sm, st, nullptr);
    case 3: return launch_lip_3(true, false, Q, sm, st, nullptr);
    case 4: return launch_lip_4(true, false, Q, sm, st, nullptr);
    case 5: return launch_lip_5(true, false, Q, sm, st, nullptr);
    case 6: return launch_lip_6(true, false, Q, sm, st, nullptr);
    }
    return hipErrorInvalidValue;
}

// res_out != null: no launch, report the resident workgroups of the solve kernel (0 for DD: no queue)
hipError_t launch(const Handle* h, bool solve, const KP& P, hipStream_t st, unsigned* res_out = nullptr)
{
    const size_t smem = smem_bytes(h, solve);
    const bool f32 = h->cfg.precision == ALIPMPC_PREC_FP32;
    if (h->cfg.variant == ALIPMPC_VARIANT_DD && res_out) {
        *res_out = 0;
        return hipSuccess;
    }
    if (h->cfg.variant == ALIPMPC_VARIANT_DD) {
        switch (h->N) {
        case 1: return launch_dd_1(solve, P, smem, st);
        case 2: return launch_dd_2(solve, P, smem, st);
        case 3: return launch_dd_3(solve, P, smem, st);
        case 4: return launch_dd_4(solve, P, smem, st);
        case 5: return launch_dd_5(solve, P, smem, st);
        case 6: return launch_dd_6(solve, P, smem, st);
        }
        return hipErrorInvalidValue;
    }
    if (!solve && h->sweep_nc >= 0) {
        if (res_out) return hipErrorInvalidValue;
        return launch_sweep(h->sweep_nc, h->cfg.variant == ALIPMPC_VARIANT_MODI, P, st);
    }
    if (solve && h->lane_nct >= 0) {
        const bool modi = h->cfg.variant == ALIPMPC_VARIANT_MODI;
        if (res_out || !P.resto_ipopt)
            return f32 ? launch_lane_f32(h->lane_nct, modi, P, st, res_out) : launch_lane_f64(h->lane_nct, modi, P, st, res_out);
        // cfg.restoration = IPOPT: the lane program solves every instance whose line searches all succeed; an instance
        // whose search fails is listed (P.redo) and solved from its start by the fp64 wave program's restoration-capable
        // work queue, on the same stream (the same queue pair: the lane kernel's last wave resets it)
        KP P1 = P;
        if (hipError_t e = redo_list(h, st, P.B, &P1.redo)) return e;
        if (hipError_t e = hipMemsetAsync(P1.redo, 0, sizeof(uint32_t), st)) return e;
        if (hipError_t e = f32 ? launch_lane_f32(h->lane_nct, modi, P1, st, nullptr)
                               : launch_lane_f64(h->lane_nct, modi, P1, st, nullptr))
            return e;
        return launch_handoff(h, P, P1.redo, st);
    }
    if (solve && f32 && P.resto_ipopt && !res_out && !P.redo) {
        // the fp32 wave program, cfg.restoration = IPOPT: the same hand-off (solve_one lists an instance whose search
        // fails).  Phase 1 of a split launch starts the list and phase 2 continues it; the fp64 work queue runs after
        // the last launch of the solve.
        KP P1 = P;
        if (hipError_t e = redo_list(h, st, P.B, &P1.redo)) return e;
        if (!P.resume)
            if (hipError_t e = hipMemsetAsync(P1.redo, 0, sizeof(uint32_t), st)) return e;
        if (hipError_t e = launch(h, true, P1, st)) return e;
        if (P.ckpt && !P.resume) return hipSuccess;
        return launch_handoff(h, P, P1.redo, st);
    }
    switch (h->N) {
    case 1: return launch_lip_1(solve, f32, P, smem, st, res_out);
    case 2: return launch_lip_2(solve, f32, P, smem, st, res_out);
    case 3: return launch_lip_3(solve, f32, P, smem, st, res_out);
    case 4: return launch_lip_4(solve, f32, P, smem, st, res_out);
    case 5: return launch_lip_5(solve, f32, P, smem, st, res_out);
    case 6: return launch_lip_6(solve, f32, P, smem, st, res_out);
    }
    return hipErrorInvalidValue;
}

// hip_stream argument -> the stream to launch on (NULL = host-pointer mode on the handle's own stream,
// ALIPMPC_STREAM_NULL = device pointers on the null stream)
hipStream_t stream_of(const Handle* h, void* hip_stream)
{
    if (!hip_stream) return h->own;
    if (hip_stream == ALIPMPC_STREAM_NULL) return nullptr;
    return (hipStream_t)hip_stream;
}

bool create_events(Handle* h)
{
    for (auto& pr : h->ev)
        for (hipEvent_t& e : pr)
            if (hipEventCreate(&e) != hipSuccess) return false;
    return true;
}

int ensure_stage(Handle* h, size_t bytes)
{
    if (h->stage_bytes >= bytes) return 0;
    if (h->stage) hipFree(h->stage);
    h->stage = nullptr;
    h->stage_bytes = 0;
    HIPCHK(h, hipMalloc(&h->stage, bytes));
    h->stage_bytes = bytes;
    return 0;
}

struct Carver {
    char* base;
    size_t off = 0;
    template <class T>
    T* take(size_t count)
    {
        off = (off + 255) & ~(size_t)255;
        T* p = reinterpret_cast<T*>(base + off);
        off += count * sizeof(T);
        return p;
    }
};

}  // namespace

extern "C" {

int alipmpc_default_cfg(int32_t variant, int32_t N, alipmpc_cfg* c)
{
    if (!c) return ALIPMPC_EINVAL;
    std::memset(c, 0, sizeof(*c));
    c->N = N;
    c->nc_max = 6;
    c->ne_max = 6;
    c->variant = variant;
    // the reference's IPOPT caps: MPC_LIP_modi.py:287 (30), MPC_LIP_sig_step.py:269 (20), MPC_DD_sig_step.py:183 (40)
    c->max_iter = variant == ALIPMPC_VARIANT_SIG_STEP ? 20 : variant == ALIPMPC_VARIANT_DD ? 40 : 30;
    c->precision = ALIPMPC_PREC_FP64;
    c->select_obs = 1;
    c->detour = 1;
    c->tol = 1e-8;
    c->acceptable_tol = 1e-6;
    c->dt = 0.4;
    c->H = 1.0;
    c->g = 9.81;
    c->leg2_max = 0.09;
    c->bvx_lo = 0.4;
    c->bvx_hi = 0.8;
    c->bvy_lo = 0.15;
    c->bvy_hi = 0.35;
    c->dtheta_max = M_PI / 16;
    c->q = 1.0;
    c->p = 0.0;
    c->r = 50.0;
    c->gamma = 0.2;
    c->s = 0.024 * 180 / M_PI;
    c->detect_r2 = 16.0;
    c->dd_t = 2.0;
    c->mu_init = 0.1;
    if (variant == ALIPMPC_VARIANT_SIG_STEP) {   // MPC_LIP_sig_step.py:38,340-353
        c->bvy_hi = 0.30;
        c->p = 2.0;
        c->r = 15.0;
        c->gamma = 0.4;
        c->s = 0.014 * 180 / M_PI;
        c->select_obs = 0;
    } else if (variant == ALIPMPC_VARIANT_DD) {  // MPC_DD_sig_step.py:33-37,323-338
        c->select_obs = 0;
        c->detour = 0;
    } else if (variant != ALIPMPC_VARIANT_MODI) {
        return ALIPMPC_EINVAL;
    }
    return ALIPMPC_OK;
}

int32_t alipmpc_rows_per_step(const alipmpc_cfg* c)
{
    if (!c) return 0;
    if (c->variant == ALIPMPC_VARIANT_DD) return c->nc_max + c->ne_max + 1;
    return 4 + c->nc_max + c->ne_max + (c->variant == ALIPMPC_VARIANT_MODI ? 1 : 0);
}

int32_t alipmpc_num_vars(const alipmpc_cfg* c)
{
    if (!c) return 0;
    return c->variant == ALIPMPC_VARIANT_DD ? 2 * c->N : 5 * c->N;
}

int alipmpc_create(const alipmpc_cfg* cfg, int device, void** handle)
{
    if (!cfg || !handle) return ALIPMPC_EINVAL;
    *handle = nullptr;
    if (cfg->N < 1 || cfg->N > ALIPMPC_MAX_N || cfg->nc_max < 0 || cfg->ne_max < 0 ||
        cfg->nc_max + cfg->ne_max > ALIPMPC_MAX_OBS || cfg->max_iter < 0 || cfg->max_iter > FILTER_CAP - 2)
        return ALIPMPC_EINVAL;
    if (cfg->precision != ALIPMPC_PREC_FP64 && cfg->precision != ALIPMPC_PREC_FP32) return ALIPMPC_EINVAL;
    if (cfg->program != ALIPMPC_PROGRAM_WAVE && cfg->program != ALIPMPC_PROGRAM_LANE) return ALIPMPC_EINVAL;
    // enum fields: callers start from alipmpc_default_cfg (a struct filled by hand must set them to a defined value)
    if (cfg->goal_singular != ALIPMPC_GOAL_SINGULAR_ZERO && cfg->goal_singular != ALIPMPC_GOAL_SINGULAR_ABORT)
        return ALIPMPC_EINVAL;
    if (cfg->restoration != ALIPMPC_RESTORATION_IPOPT && cfg->restoration != ALIPMPC_RESTORATION_SUBSTITUTE)
        return ALIPMPC_EINVAL;
    // fp32 arithmetic is implemented for the LIP solve kernels (modi, sig_step)
    if (cfg->precision == ALIPMPC_PREC_FP32 && cfg->variant == ALIPMPC_VARIANT_DD) return ALIPMPC_EUNSUPPORTED;
    if (cfg->variant != ALIPMPC_VARIANT_MODI && cfg->variant != ALIPMPC_VARIANT_SIG_STEP &&
        cfg->variant != ALIPMPC_VARIANT_DD)
        return ALIPMPC_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return ALIPMPC_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return ALIPMPC_ENODEV;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return ALIPMPC_ENODEV;
    Handle* h = new Handle();
    h->cfg = *cfg;
    if (cfg->precision == ALIPMPC_PREC_FP32 && cfg->tol == 1e-8 && cfg->acceptable_tol == 1e-6) {
        // the fp64 defaults are below fp32 resolution: use the horizon-aware fp32 defaults (the ctypes
        // layer's FP32_TOL*); N > 3 decision-space gradients grow through A^k and lift the fp32 floor
        h->cfg.tol = cfg->N > 3 ? 3e-4 : 1e-4;
        h->cfg.acceptable_tol = cfg->N > 3 ? 3e-3 : 1e-3;
    }
    h->device = device;
    h->N = cfg->N;
    h->n = 3 * cfg->N;
    h->NG = 8 * (cfg->N + 1);
    h->NCP = 16 * ((h->n + 15) / 16);
    h->NCPU = 16 * ((5 * cfg->N + 15) / 16);
    h->rps = alipmpc_rows_per_step(cfg);
    h->m_max = cfg->N * h->rps;
    h->mr4 = (h->m_max + 3) & ~3;
    if (cfg->variant == ALIPMPC_VARIANT_DD) {
        // DD solve rows per step: cbf slots, v +- s w, v bound, w bound; + N objective rows; whole
        // 64-lane row groups (dd_solve_kernel<N, RPL>)
        h->rps_s = cfg->nc_max + cfg->ne_max + 4;
        h->m_s = cfg->N * h->rps_s;
        h->mr4_s = (h->m_s + 3) & ~3;
        const int rpl = (h->mr4_s + cfg->N + WAVE - 1) / WAVE;
        h->mo4 = rpl <= 3 ? WAVE * rpl : 1 << 20;
    } else {
        h->rps_s = h->rps + (cfg->variant == ALIPMPC_VARIANT_MODI ? 1 : 0);   // f_en -> two smooth rows
        h->m_s = cfg->N * h->rps_s;
        h->mr4_s = (h->m_s + 3) & ~3;
        // + the objective pseudo-rows of the solve kernel, rounded up to the compiled J-layout size (4 KSM)
        h->mo4 = 4 * ksm_of(h->mr4_s + 4 * ((cfg->N + 3) / 4));
    }
    if (h->mr4 > MAX_ROWS || h->mo4 > MAX_ROWS + 64) {
        delete h;
        return ALIPMPC_EINVAL;
    }
    if (hipSetDevice(device) != hipSuccess) {
        delete h;
        return ALIPMPC_ENODEV;
    }
    std::vector<double> Gp, Ep, Gu, Eu;
    build_tables(*cfg, h->NCP, h->NCPU, Gp, Ep, Gu, Eu);
    auto up = [](double** d, const std::vector<double>& v) {
        return hipMalloc(d, v.size() * sizeof(double)) == hipSuccess &&
               hipMemcpy(*d, v.data(), v.size() * sizeof(double), hipMemcpyHostToDevice) == hipSuccess;
    };
    if (!up(&h->dGp, Gp) || !up(&h->dEp, Ep) || !up(&h->dGu, Gu) || !up(&h->dEu, Eu) ||
        hipMalloc(&h->dq, 2 * (Handle::NQ + Handle::MAXG) * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&h->dlk, alip::lane::LK_BUF * sizeof(double)) != hipSuccess ||
        hipMalloc(&h->dlkf, alip::lane::LK_BUF * sizeof(float)) != hipSuccess ||
        hipMemset(h->dq, 0, 2 * (Handle::NQ + Handle::MAXG) * sizeof(uint32_t)) != hipSuccess ||
        hipStreamCreateWithFlags(&h->own, hipStreamNonBlocking) != hipSuccess ||
        !create_events(h)) {
        alipmpc_destroy(h);
        return ALIPMPC_EHIP;
    }
    {
        double lk[alip::lane::LK_BUF];
        float lkf[alip::lane::LK_BUF];
        lane_constants(h->cfg, lk);
        for (int i = 0; i < alip::lane::LK_BUF; ++i) lkf[i] = (float)lk[i];
        if (hipMemcpy(h->dlk, lk, sizeof(lk), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(h->dlkf, lkf, sizeof(lkf), hipMemcpyHostToDevice) != hipSuccess) {
            alipmpc_destroy(h);
            return ALIPMPC_EHIP;
        }
        // the eval hook's sweep kernel: N = 3, circle slots only (ALIPMPC_EVAL_KERNEL=group selects eval_kernel,
        // for A/B and the bit-identity test)
        const char* ek = std::getenv("ALIPMPC_EVAL_KERNEL");
        if (h->cfg.variant != ALIPMPC_VARIANT_DD && h->cfg.N == 3 && h->cfg.ne_max == 0 && h->cfg.nc_max <= 6 &&
            !(ek && std::strcmp(ek, "group") == 0))
            h->sweep_nc = h->cfg.nc_max;
        {   // split launch of one-wave-per-instance batches (ALIPMPC_SPLIT_IT=0 turns it off)
            const char* se = std::getenv("ALIPMPC_SPLIT_IT");
            h->split_it = se ? std::atoi(se)
                             : (cfg->restoration == ALIPMPC_RESTORATION_IPOPT ? SPLIT_IT_DEFAULT_RESTO : SPLIT_IT_DEFAULT);
            if (h->split_it < 0 || h->split_it >= h->cfg.max_iter) h->split_it = 0;
            auto env_int = [](const char* name, int dflt) {
                const char* t = std::getenv(name);
                return t ? std::max(0, std::atoi(t)) : dflt;
            };
            h->split_tr = env_int("ALIPMPC_SPLIT_TR", SPLIT_TR_DEFAULT);
            h->cl_split_it = env_int("ALIPMPC_CL_SPLIT_IT", CL_SPLIT_IT_DEFAULT);
            if (h->cl_split_it >= h->cfg.max_iter) h->cl_split_it = 0;
            h->cl_split_tr = env_int("ALIPMPC_CL_SPLIT_TR", CL_SPLIT_TR_DEFAULT);
        }
        if (h->cfg.program == ALIPMPC_PROGRAM_LANE) {
            h->lane_nct = lane_slots_for(h->cfg);
            if (h->lane_nct < 0) {
                alipmpc_destroy(h);
                return ALIPMPC_EUNSUPPORTED;
            }
        }
    }
    // (fp32 with cfg.restoration = IPOPT hands instances to the fp64 wave program: its workspace must fit as well)
    const bool handoff = cfg->variant != ALIPMPC_VARIANT_DD && cfg->restoration == ALIPMPC_RESTORATION_IPOPT &&
                         (cfg->precision == ALIPMPC_PREC_FP32 || h->lane_nct >= 0);
    if (smem_bytes(h, true) > 160 * 1024 || smem_bytes(h, false) > 160 * 1024 ||
        (handoff && smem_bytes(h, true, 1) > 160 * 1024)) {
        alipmpc_destroy(h);
        return ALIPMPC_EUNSUPPORTED;
    }
    // team records need the team-capable build's TEAM_WAVES workspaces in one workgroup: without room, no trial cut
    if (cfg->variant != ALIPMPC_VARIANT_DD && cfg->precision != ALIPMPC_PREC_FP32 && h->lane_nct < 0) {
        size_t st_ = 0;
        switch (h->N) {
#define TSCASE(NN) \
    case NN: st_ = team_smem<NN, double>(smem_bytes(h, true)); break;
            TSCASE(1) TSCASE(2) TSCASE(3) TSCASE(4) TSCASE(5) TSCASE(6)
#undef TSCASE
        }
        if (st_ > 160 * 1024) h->split_tr = h->cl_split_tr = 0;
    }
    *handle = h;
    return ALIPMPC_OK;
}

// A wave-program solve whose batch fits the resident slots (one wave per instance) runs as a SPLIT launch: phase 1
// solves every instance for up to split_it iterations; an instance still running then writes its loop state to a
// record and stops; phase 2 resumes those instances, one wave each.  The long instances (cfg2: 12 % run to the
// 30-iteration cap) otherwise finish at the pace of the busiest SIMDs, which hold two or three of them
// among their four waves; in phase 2 they are few enough for a SIMD each.  Every instance executes the same
// arithmetic either way (the record holds its exact loop state): same bits (test_split_launch_bit_identical).
// whether a solve of B instances with these cuts runs as a split launch (launch_solve and alipmpc_solve_launches share
// it): the wave program (not DD), an iteration cut or — fp64, the team-capable build — a trial cut, B within the slots
static bool split_form(const Handle* h, long long B, int split_it, int split_tr, long long slots)
{
    const alipmpc_cfg& cf = h->cfg;
    if (cf.precision == ALIPMPC_PREC_FP32) split_tr = 0;   // (the team-capable build is fp64 only)
    return cf.variant != ALIPMPC_VARIANT_DD && h->lane_nct < 0 && (split_it > 0 || split_tr > 0) && B >= 2 &&
           B <= slots;
}

// the stream's record buffer (Handle::split), sized for `slots` instances; nullptr: run the one-phase form
static void* split_buffer(Handle* h, hipStream_t st, size_t need, hipError_t& err)
{
    err = hipSuccess;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess) return nullptr;
    const bool capturing = cs != hipStreamCaptureStatusNone;
    std::lock_guard<std::mutex> lk(h->split_mtx);
    auto it = h->split.find(st);
    if (it == h->split.end()) {
        if (capturing) return nullptr;   // no allocation inside a capture: the one-phase form
        // every buffer is kept until alipmpc_destroy (an eviction's hipFree synchronised the device and
        // could free a buffer another thread had just been handed); a stream beyond SPLIT_STREAMS runs the one-phase
        // form, which computes the same bits
        // (the closed loop's own group streams do not count: ADVICE r5 — cycling user streams would otherwise leave
        // its episode groups on the one-phase form)
        bool group = false;
        for (int g = 0; g < Handle::MAXG; ++g) group |= st != nullptr && st == h->gst[g];
        size_t users = 0;
        for (auto& kv : h->split) {
            bool gk = false;
            for (int g = 0; g < Handle::MAXG; ++g) gk |= kv.first != nullptr && kv.first == h->gst[g];
            users += gk ? 0 : 1;
        }
        if (!group && users >= Handle::SPLIT_STREAMS) return nullptr;
        Handle::SplitBuf sb;
        if ((err = hipMalloc(&sb.p, need)) != hipSuccess) return nullptr;
        sb.bytes = need;
        it = h->split.emplace(st, sb).first;
    }
    if (it->second.bytes < need) return nullptr;   // (sized for the slots: does not happen)
    return it->second.p;
}

static hipError_t launch_solve(Handle* h, const KP& P, hipStream_t st, int split_it, int split_tr)
{
    const alipmpc_cfg& cf = h->cfg;
    if (cf.precision == ALIPMPC_PREC_FP32) split_tr = 0;   // (the team-capable build is fp64 only)
    if (!split_form(h, P.B, split_it, split_tr, 1ll << 62) || P.order) return launch(h, true, P, st);
    unsigned res = 0;
    if (hipError_t e = launch(h, true, P, st, &res)) return e;
    const long long slots = (long long)res * WAVES_PER_BLOCK;
    if (slots < P.B) return launch(h, true, P, st);   // the work-queue form
    // records for the slots, not for this B: the buffer of a stream never changes size
    const size_t rec_bytes = ((size_t)slots * ckpt_doubles(h->mo4) * sizeof(double) + 255) & ~(size_t)255;
    const size_t hdr = (size_t)cont_hdr(slots);
    const size_t need = rec_bytes + (hdr + (size_t)slots) * sizeof(uint32_t);
    hipError_t berr = hipSuccess;
    void* buf = split_buffer(h, st, need, berr);
    if (berr != hipSuccess) return berr;
    if (!buf) return launch(h, true, P, st);
    uint32_t* cont = reinterpret_cast<uint32_t*>((char*)buf + rec_bytes);
    if (hipError_t e = hipMemsetAsync(cont, 0, hdr * sizeof(uint32_t), st)) return e;
    const int team = split_tr > 0 ? (int)std::min<long long>(P.B, TEAM_CAP) : 0;
    KP P1 = P;
    P1.ckpt_it = split_it > 0 ? split_it : 0;
    P1.ckpt_tr = split_tr;
    P1.team = team;
    P1.ckpt = (double*)buf;
    P1.cont = cont;
    if (hipError_t e = launch(h, true, P1, st)) return e;
    KP P2 = P;   // single records, and team records
    P2.resume = 1;
    P2.team = team;
    P2.ckpt = (double*)buf;
    P2.cont = cont;
    return launch(h, true, P2, st);
}

static int run_batch(Handle* h, bool solve, int64_t B, const double* x0, const double* goal, const int8_t* leg,
                     const double* cir, const int32_t* nc, const double* elp, const int32_t* ne, const double* u0,
                     const double* last_u, double* u_out, double* foot_out, double* x_pred, int32_t* status, int32_t* iters, double* f,
                     double* grad, double* c, double* J, double* cl, double* cu, double* goal_eff, int8_t* row_active,
                     void* hip_stream)
{
    if (!h) return ALIPMPC_EINVAL;
    if (B < 0) return fail(h, ALIPMPC_EINVAL, "B < 0");
    if (B == 0) return ALIPMPC_OK;
    const alipmpc_cfg& cf = h->cfg;
    const bool dd = cf.variant == ALIPMPC_VARIANT_DD;
    if (!x0 || !goal || (!leg && !dd) || !nc || !u0 || (cf.nc_max > 0 && !cir) || (cf.ne_max > 0 && (!elp || !ne)))
        return fail(h, ALIPMPC_EINVAL, "missing input pointer");
    if (solve && !u_out) return fail(h, ALIPMPC_EINVAL, "u_out is required");
    if (solve && B >= (int64_t)1 << 31) return fail(h, ALIPMPC_EINVAL, "B >= 2^31 (32-bit work-queue counter)");
    HIPCHK(h, hipSetDevice(h->device));
    // host-facing u: the reference's 5N-vector (LIP) / 2N controls (DD); state dimension 5 / 3
    const int N = h->N, n = dd ? 2 * N : 5 * N, sd = dd ? 3 : 5;
    const size_t mm_ = (size_t)h->m_max;
    KP P = make_kp(h, B, solve);
    hipStream_t st = stream_of(h, hip_stream);
    if (hip_stream) {
        P.x0 = x0; P.goal = goal; P.leg = leg; P.cir = cir; P.nc = nc; P.elp = elp; P.ne = ne; P.u0 = u0;
        P.last_u = last_u;
        P.u_out = u_out; P.foot_out = foot_out; P.x_pred = x_pred; P.status = status; P.iters = iters;
        P.f_out = f; P.grad_out = grad; P.c_out = c; P.J_out = J; P.cl_out = cl; P.cu_out = cu;
        P.goal_eff_out = goal_eff; P.active_out = row_active;
        const int ei = h->evi;
        h->evi = (ei + 1) % Handle::NEV;
        HIPCHK(h, hipEventRecord(h->ev[ei][0], st));
        HIPCHK(h, solve ? launch_solve(h, P, st, h->split_it, h->split_tr) : launch(h, false, P, st));
        HIPCHK(h, hipEventRecord(h->ev[ei][1], st));
        h->evlast = ei;
        h->timed = true;
        return ALIPMPC_OK;
    }
    // host pointers: stage through the handle's device workspace (only the regions this call uses: the
    // solve outputs for a solve, the eval outputs for an eval, J only when it is requested)
    const size_t Bz = (size_t)B;
    struct Stage {
        double *x0, *goal, *cir, *elp, *u0, *lu, *u, *foot, *xp, *f, *g, *c, *J, *cl, *cu, *ge;
        int8_t *leg, *ra;
        int32_t *nc, *ne, *st, *it;
    };
    auto carve = [&](Carver& cv) {
        Stage z{};
        z.x0 = cv.take<double>(Bz * sd);
        z.goal = cv.take<double>(Bz * 2);
        z.leg = cv.take<int8_t>(Bz);
        z.cir = cv.take<double>(Bz * 3 * cf.nc_max);
        z.nc = cv.take<int32_t>(Bz);
        z.elp = cv.take<double>(Bz * 5 * cf.ne_max);
        z.ne = cv.take<int32_t>(Bz);
        z.u0 = cv.take<double>(Bz * n);
        z.lu = cv.take<double>(Bz * 2);
        if (solve) {
            z.u = cv.take<double>(Bz * n);
            z.foot = cv.take<double>(Bz * 3);
            z.xp = cv.take<double>(Bz * sd * N);
            z.st = cv.take<int32_t>(Bz);
            z.it = cv.take<int32_t>(Bz);
        } else {
            z.f = cv.take<double>(Bz);
            z.g = cv.take<double>(Bz * n);
            z.c = cv.take<double>(Bz * mm_);
            if (J) z.J = cv.take<double>(Bz * mm_ * n);
            z.cl = cv.take<double>(Bz * mm_);
            z.cu = cv.take<double>(Bz * mm_);
            z.ge = cv.take<double>(Bz * 2);
            z.ra = cv.take<int8_t>(Bz * mm_);
        }
        return z;
    };
    size_t need = 0;
    {
        Carver cv{nullptr};
        carve(cv);
        need = cv.off + 256;
    }
    if (int e = ensure_stage(h, need)) return e;
    Carver cv{(char*)h->stage};
    const Stage z = carve(cv);
    double *d_x0 = z.x0, *d_goal = z.goal, *d_cir = z.cir, *d_elp = z.elp, *d_u0 = z.u0, *d_lu = z.lu;
    double *d_u = z.u, *d_foot = z.foot, *d_xp = z.xp, *d_f = z.f, *d_g = z.g, *d_c = z.c, *d_J = z.J;
    double *d_cl = z.cl, *d_cu = z.cu, *d_ge = z.ge;
    int8_t *d_leg = z.leg, *d_ra = z.ra;
    int32_t *d_nc = z.nc, *d_ne = z.ne, *d_st = z.st, *d_it = z.it;
    auto h2d = [&](void* d, const void* s, size_t bytes) { return hipMemcpyAsync(d, s, bytes, hipMemcpyHostToDevice, st); };
    auto d2h = [&](void* d, const void* s, size_t bytes) { return hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToHost, st); };
    HIPCHK(h, h2d(d_x0, x0, Bz * sd * 8));
    HIPCHK(h, h2d(d_goal, goal, Bz * 2 * 8));
    if (leg) HIPCHK(h, h2d(d_leg, leg, Bz));
    if (cf.nc_max) HIPCHK(h, h2d(d_cir, cir, Bz * 3 * cf.nc_max * 8));
    HIPCHK(h, h2d(d_nc, nc, Bz * 4));
    if (cf.ne_max) {
        HIPCHK(h, h2d(d_elp, elp, Bz * 5 * cf.ne_max * 8));
        HIPCHK(h, h2d(d_ne, ne, Bz * 4));
    }
    HIPCHK(h, h2d(d_u0, u0, Bz * n * 8));
    if (last_u) HIPCHK(h, h2d(d_lu, last_u, Bz * 2 * 8));
    P.last_u = last_u ? d_lu : nullptr;
    P.x0 = d_x0; P.goal = d_goal; P.leg = leg ? d_leg : nullptr; P.cir = d_cir; P.nc = d_nc;
    P.elp = cf.ne_max ? d_elp : nullptr; P.ne = cf.ne_max ? d_ne : nullptr; P.u0 = d_u0;
    if (solve) {
        P.u_out = d_u; P.foot_out = d_foot; P.x_pred = d_xp; P.status = d_st; P.iters = d_it;
    } else {
        P.f_out = d_f; P.grad_out = d_g; P.c_out = d_c; P.J_out = J ? d_J : nullptr; P.cl_out = d_cl; P.cu_out = d_cu;
        P.goal_eff_out = d_ge; P.active_out = d_ra;
    }
    const int ei = h->evi;
    h->evi = (ei + 1) % Handle::NEV;
    HIPCHK(h, hipEventRecord(h->ev[ei][0], st));
    HIPCHK(h, solve ? launch_solve(h, P, st, h->split_it, h->split_tr) : launch(h, false, P, st));
    HIPCHK(h, hipEventRecord(h->ev[ei][1], st));
    h->evlast = ei;
    h->timed = true;
    if (solve) {
        HIPCHK(h, d2h(u_out, d_u, Bz * n * 8));
        if (foot_out) HIPCHK(h, d2h(foot_out, d_foot, Bz * 3 * 8));
        if (x_pred) HIPCHK(h, d2h(x_pred, d_xp, Bz * sd * N * 8));
        if (status) HIPCHK(h, d2h(status, d_st, Bz * 4));
        if (iters) HIPCHK(h, d2h(iters, d_it, Bz * 4));
    } else {
        if (f) HIPCHK(h, d2h(f, d_f, Bz * 8));
        if (grad) HIPCHK(h, d2h(grad, d_g, Bz * n * 8));
        if (c) HIPCHK(h, d2h(c, d_c, Bz * mm_ * 8));
        if (J) HIPCHK(h, d2h(J, d_J, Bz * mm_ * n * 8));
        if (cl) HIPCHK(h, d2h(cl, d_cl, Bz * mm_ * 8));
        if (cu) HIPCHK(h, d2h(cu, d_cu, Bz * mm_ * 8));
        if (goal_eff) HIPCHK(h, d2h(goal_eff, d_ge, Bz * 2 * 8));
        if (row_active) HIPCHK(h, d2h(row_active, d_ra, Bz * mm_));
    }
    HIPCHK(h, hipStreamSynchronize(st));
    return ALIPMPC_OK;
}

int alipmpc_solve_batch(void* handle, int64_t B, const double* x0, const double* goal, const int8_t* leg,
                        const double* cir, const int32_t* nc, const double* elp, const int32_t* ne, const double* u0,
                        const double* last_u, double* u_out, double* foot_out, double* x_pred, int32_t* status,
                        int32_t* iters, void* hip_stream)
{
    return run_batch((Handle*)handle, true, B, x0, goal, leg, cir, nc, elp, ne, u0, last_u, u_out, foot_out, x_pred, status,
                     iters, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, hip_stream);
}

int alipmpc_eval_batch(void* handle, int64_t B, const double* x0, const double* goal, const int8_t* leg,
                       const double* cir, const int32_t* nc, const double* elp, const int32_t* ne, const double* u,
                       const double* last_u, double* f, double* grad, double* c, double* J, double* cl, double* cu,
                       double* goal_eff, int8_t* row_active, void* hip_stream)
{
    return run_batch((Handle*)handle, false, B, x0, goal, leg, cir, nc, elp, ne, u, last_u, nullptr, nullptr, nullptr,
                     nullptr, nullptr, f, grad, c, J, cl, cu, goal_eff, row_active, hip_stream);
}

int alipmpc_rollout_batch(void* handle, int64_t B, int32_t S, const double* x0, const double* goal, const int8_t* leg,
                          const double* cir, const int32_t* nc, const double* elp, const int32_t* ne, const double* u0,
                          const double* last_u, double* foot_traj, double* x_traj, int32_t* status_traj,
                          int32_t* iters_traj, int32_t* steps_to_goal, double* u_traj, void* hip_stream)
{
    Handle* h = (Handle*)handle;
    if (!h) return ALIPMPC_EINVAL;
    if (B < 0 || S < 0) return fail(h, ALIPMPC_EINVAL, "B < 0 or S < 0");
    if (B == 0 || S == 0) return ALIPMPC_OK;
    const alipmpc_cfg& cf = h->cfg;
    const bool dd = cf.variant == ALIPMPC_VARIANT_DD;
    if (!x0 || !goal || (!leg && !dd) || !nc || !u0 || (cf.nc_max > 0 && !cir) || (cf.ne_max > 0 && (!elp || !ne)))
        return fail(h, ALIPMPC_EINVAL, "missing input pointer");
    HIPCHK(h, hipSetDevice(h->device));
    const int N = h->N, n = dd ? 2 * N : 5 * N, sd = dd ? 3 : 5;
    const size_t Bz = (size_t)B, Sz = (size_t)S;
    hipStream_t st = stream_of(h, hip_stream);
    const bool host = hip_stream == nullptr;   // ALIPMPC_STREAM_NULL: device pointers, null stream
    // working set (+ staged inputs / outputs for host-pointer calls)
    auto layout = [&](Carver& cv, bool take_io) {
        struct L {
            double *x, *u0, *lu, *u, *foot, *xp;
            int8_t* leg;
            int32_t *st, *it;
            uint8_t* act;
            double *goal, *cir, *elp, *ft, *xt, *ut;
            int32_t *nc, *ne, *stt, *itt, *sg;
        } l{};
        l.x = cv.take<double>(Bz * sd); l.u0 = cv.take<double>(Bz * n); l.lu = cv.take<double>(Bz * 2);
        l.u = cv.take<double>(Bz * n); l.foot = cv.take<double>(Bz * 3); l.xp = cv.take<double>(Bz * N * sd);
        l.leg = cv.take<int8_t>(Bz); l.st = cv.take<int32_t>(Bz); l.it = cv.take<int32_t>(Bz);
        l.act = cv.take<uint8_t>(Bz);
        if (take_io) {
            l.goal = cv.take<double>(Bz * 2); l.cir = cv.take<double>(Bz * 3 * cf.nc_max);
            l.elp = cv.take<double>(Bz * 5 * cf.ne_max); l.nc = cv.take<int32_t>(Bz); l.ne = cv.take<int32_t>(Bz);
            l.ft = cv.take<double>(Bz * Sz * 3); l.xt = cv.take<double>(Bz * (Sz + 1) * sd);
            l.stt = cv.take<int32_t>(Bz * Sz); l.itt = cv.take<int32_t>(Bz * Sz); l.sg = cv.take<int32_t>(Bz);
            if (u_traj) l.ut = cv.take<double>(Bz * Sz * n);
        }
        return l;
    };
    size_t need;
    {
        Carver cv{nullptr};
        layout(cv, host);
        need = cv.off + 256;
    }
    if (h->rstage_bytes < need) {
        if (h->rstage) hipFree(h->rstage);
        h->rstage = nullptr;
        h->rstage_bytes = 0;
        HIPCHK(h, hipMalloc(&h->rstage, need));
        h->rstage_bytes = need;
    }
    Carver cv{(char*)h->rstage};
    auto l = layout(cv, host);
    const hipMemcpyKind in_kind = host ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
    HIPCHK(h, hipMemcpyAsync(l.x, x0, Bz * sd * 8, in_kind, st));
    HIPCHK(h, hipMemcpyAsync(l.u0, u0, Bz * n * 8, in_kind, st));
    if (leg) HIPCHK(h, hipMemcpyAsync(l.leg, leg, Bz, in_kind, st));
    if (last_u)
        HIPCHK(h, hipMemcpyAsync(l.lu, last_u, Bz * 2 * 8, in_kind, st));
    else
        HIPCHK(h, hipMemsetAsync(l.lu, 0, Bz * 2 * 8, st));
    const double *d_goal = goal, *d_cir = cir, *d_elp = elp;
    const int32_t *d_nc = nc, *d_ne = ne;
    double *d_ft = foot_traj, *d_xt = x_traj, *d_ut = u_traj;
    int32_t *d_stt = status_traj, *d_itt = iters_traj, *d_sg = steps_to_goal;
    if (host) {
        HIPCHK(h, hipMemcpyAsync(l.goal, goal, Bz * 2 * 8, hipMemcpyHostToDevice, st));
        if (cf.nc_max) HIPCHK(h, hipMemcpyAsync(l.cir, cir, Bz * 3 * cf.nc_max * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(l.nc, nc, Bz * 4, hipMemcpyHostToDevice, st));
        if (cf.ne_max) {
            HIPCHK(h, hipMemcpyAsync(l.elp, elp, Bz * 5 * cf.ne_max * 8, hipMemcpyHostToDevice, st));
            HIPCHK(h, hipMemcpyAsync(l.ne, ne, Bz * 4, hipMemcpyHostToDevice, st));
        }
        d_goal = l.goal; d_cir = l.cir; d_nc = l.nc;
        d_elp = cf.ne_max ? l.elp : nullptr;
        d_ne = cf.ne_max ? l.ne : nullptr;
        d_ft = foot_traj ? l.ft : nullptr; d_xt = x_traj ? l.xt : nullptr;
        d_stt = status_traj ? l.stt : nullptr; d_itt = iters_traj ? l.itt : nullptr;
        d_sg = steps_to_goal ? l.sg : nullptr;
        d_ut = u_traj ? l.ut : nullptr;
    }
    const unsigned g1 = (unsigned)((B + 255) / 256);
    hipLaunchKernelGGL(rollout_init_kernel, dim3(g1), dim3(256), 0, st, (long long)B, (int)S, sd, (const double*)l.x,
                       d_xt, l.act, d_sg);
    HIPCHK(h, hipGetLastError());
    KP P = make_kp(h, B, true);
    P.goal = d_goal; P.cir = d_cir; P.nc = d_nc; P.elp = d_elp; P.ne = d_ne;
    P.x0 = l.x; P.leg = dd ? nullptr : l.leg; P.u0 = l.u0; P.last_u = dd ? l.lu : nullptr; P.active = l.act;
    P.u_out = l.u; P.foot_out = l.foot; P.x_pred = l.xp; P.status = l.st; P.iters = l.it;
    AdvP A;
    std::memset(&A, 0, sizeof(A));
    A.B = B; A.S = S; A.N = N; A.sd = sd; A.n = n; A.variant = cf.variant; A.goal = d_goal;
    A.x = l.x; A.u0 = l.u0; A.leg = l.leg; A.last_u = l.lu; A.u = l.u; A.foot = l.foot; A.x_pred = l.xp;
    A.status = l.st; A.iters = l.it; A.active = l.act;
    A.foot_traj = d_ft; A.x_traj = d_xt; A.status_traj = d_stt; A.iters_traj = d_itt; A.steps_to_goal = d_sg;
    A.u_traj = d_ut;
    const int ei = h->evi;
    h->evi = (ei + 1) % Handle::NEV;
    HIPCHK(h, hipEventRecord(h->ev[ei][0], st));
    for (int t = 0; t < S; ++t) {
        HIPCHK(h, launch(h, true, P, st));
        A.t = t;
        hipLaunchKernelGGL(advance_kernel, dim3(g1), dim3(256), 0, st, A);
        HIPCHK(h, hipGetLastError());
    }
    HIPCHK(h, hipEventRecord(h->ev[ei][1], st));
    h->evlast = ei;
    h->timed = true;
    if (host) {
        if (foot_traj) HIPCHK(h, hipMemcpyAsync(foot_traj, l.ft, Bz * Sz * 3 * 8, hipMemcpyDeviceToHost, st));
        if (x_traj) HIPCHK(h, hipMemcpyAsync(x_traj, l.xt, Bz * (Sz + 1) * sd * 8, hipMemcpyDeviceToHost, st));
        if (status_traj) HIPCHK(h, hipMemcpyAsync(status_traj, l.stt, Bz * Sz * 4, hipMemcpyDeviceToHost, st));
        if (iters_traj) HIPCHK(h, hipMemcpyAsync(iters_traj, l.itt, Bz * Sz * 4, hipMemcpyDeviceToHost, st));
        if (steps_to_goal) HIPCHK(h, hipMemcpyAsync(steps_to_goal, l.sg, Bz * 4, hipMemcpyDeviceToHost, st));
        if (u_traj) HIPCHK(h, hipMemcpyAsync(u_traj, l.ut, Bz * Sz * n * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
    }
    return ALIPMPC_OK;
}

int alipmpc_closed_loop_batch(void* handle, int64_t B, int32_t S, int32_t f_cyc, double kick, uint64_t seed,
                              const double* x0, const double* foot0, const double* goal, const int8_t* leg,
                              const double* cir, const int32_t* nc, const double* elp, const int32_t* ne,
                              double* foot_traj, double* x_traj, double* hd_traj, int32_t* status_traj,
                              int32_t* iters_traj, int32_t* steps_to_goal, double* action_traj, void* hip_stream)
{
    Handle* h = (Handle*)handle;
    if (!h) return ALIPMPC_EINVAL;
    const alipmpc_cfg& cf = h->cfg;
    if (cf.variant == ALIPMPC_VARIANT_DD) return fail(h, ALIPMPC_EUNSUPPORTED, "closed loop: LIP variants only");
    if (B < 0 || S < 0 || f_cyc < 1 || !(kick >= 0)) return fail(h, ALIPMPC_EINVAL, "B, S < 0, f_cyc < 1 or kick < 0");
    if (B == 0 || S == 0) return ALIPMPC_OK;
    if (!x0 || !foot0 || !goal || !leg || !nc || (cf.nc_max > 0 && !cir) || (cf.ne_max > 0 && (!elp || !ne)))
        return fail(h, ALIPMPC_EINVAL, "missing input pointer");
    HIPCHK(h, hipSetDevice(h->device));
    const int N = h->N, n = 5 * N;
    const size_t Bz = (size_t)B, Sz = (size_t)S, Fz = (size_t)f_cyc;
    hipStream_t st = stream_of(h, hip_stream);
    const bool host = hip_stream == nullptr;
    auto layout = [&](Carver& cv, bool take_io) {
        struct L {
            double *x, *pst, *hdv, *mhd, *plan, *xs, *u0, *u, *foot, *xp;
            int8_t *leg, *sleg;
            uint8_t *flags, *act;
            int32_t *st, *it, *ord;
            double *goal, *cir, *elp, *ft, *xt, *hd, *actd;
            int32_t *nc, *ne, *stt, *itt, *sg;
            double *vdes, *pose0;
        } l{};
        l.vdes = cv.take<double>(Bz * 2); l.pose0 = cv.take<double>(Bz * 3);
        l.x = cv.take<double>(Bz * 5); l.pst = cv.take<double>(Bz * 2); l.hdv = cv.take<double>(Bz * 4);
        l.mhd = cv.take<double>(Bz * 3); l.plan = cv.take<double>(Bz * n); l.xs = cv.take<double>(Bz * 5);
        l.u0 = cv.take<double>(Bz * n); l.u = cv.take<double>(Bz * n); l.foot = cv.take<double>(Bz * 3);
        l.xp = cv.take<double>(Bz * n); l.leg = cv.take<int8_t>(Bz); l.sleg = cv.take<int8_t>(Bz);
        l.flags = cv.take<uint8_t>(Bz); l.act = cv.take<uint8_t>(Bz); l.st = cv.take<int32_t>(Bz);
        l.it = cv.take<int32_t>(Bz); l.ord = cv.take<int32_t>(Bz);
        if (take_io) {
            l.goal = cv.take<double>(Bz * 2); l.cir = cv.take<double>(Bz * 3 * cf.nc_max);
            l.elp = cv.take<double>(Bz * 5 * cf.ne_max); l.nc = cv.take<int32_t>(Bz); l.ne = cv.take<int32_t>(Bz);
            l.ft = cv.take<double>(Bz * Sz * 3); l.xt = cv.take<double>(Bz * (Sz + 1) * 5);
            l.hd = cv.take<double>(Bz * Sz * 2); l.stt = cv.take<int32_t>(Bz * Sz * Fz);
            l.itt = cv.take<int32_t>(Bz * Sz * Fz); l.sg = cv.take<int32_t>(Bz);
            if (action_traj) l.actd = cv.take<double>(Bz * Sz * Fz * 8);
        }
        return l;
    };
    size_t need;
    {
        Carver cv{nullptr};
        layout(cv, host);
        need = cv.off + 256;
    }
    if (h->rstage_bytes < need) {
        if (h->rstage) hipFree(h->rstage);
        h->rstage = nullptr;
        h->rstage_bytes = 0;
        HIPCHK(h, hipMalloc(&h->rstage, need));
        h->rstage_bytes = need;
    }
    Carver cv{(char*)h->rstage};
    auto l = layout(cv, host);
    const hipMemcpyKind in_kind = host ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
    HIPCHK(h, hipMemcpyAsync(l.x, x0, Bz * 5 * 8, in_kind, st));
    HIPCHK(h, hipMemcpyAsync(l.pst, foot0, Bz * 2 * 8, in_kind, st));
    HIPCHK(h, hipMemcpyAsync(l.leg, leg, Bz, in_kind, st));
    const double *d_goal = goal, *d_cir = cir, *d_elp = elp;
    const int32_t *d_nc = nc, *d_ne = ne;
    double *d_ft = foot_traj, *d_xt = x_traj, *d_hd = hd_traj;
    int32_t *d_stt = status_traj, *d_itt = iters_traj, *d_sg = steps_to_goal;
    double* d_act = action_traj;
    if (host) {
        HIPCHK(h, hipMemcpyAsync(l.goal, goal, Bz * 2 * 8, hipMemcpyHostToDevice, st));
        if (cf.nc_max) HIPCHK(h, hipMemcpyAsync(l.cir, cir, Bz * 3 * cf.nc_max * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(l.nc, nc, Bz * 4, hipMemcpyHostToDevice, st));
        if (cf.ne_max) {
            HIPCHK(h, hipMemcpyAsync(l.elp, elp, Bz * 5 * cf.ne_max * 8, hipMemcpyHostToDevice, st));
            HIPCHK(h, hipMemcpyAsync(l.ne, ne, Bz * 4, hipMemcpyHostToDevice, st));
        }
        d_goal = l.goal; d_cir = l.cir; d_nc = l.nc;
        d_elp = cf.ne_max ? l.elp : nullptr;
        d_ne = cf.ne_max ? l.ne : nullptr;
        d_ft = foot_traj ? l.ft : nullptr; d_xt = x_traj ? l.xt : nullptr; d_hd = hd_traj ? l.hd : nullptr;
        d_stt = status_traj ? l.stt : nullptr; d_itt = iters_traj ? l.itt : nullptr;
        d_sg = steps_to_goal ? l.sg : nullptr;
        d_act = action_traj ? l.actd : nullptr;
    }
    CLP C;
    std::memset(&C, 0, sizeof(C));
    C.B = B; C.S = S; C.f = f_cyc; C.variant = cf.variant; C.N = N; C.kick = kick; C.seed = (unsigned long long)seed;
    C.goal = d_goal; C.x = l.x; C.pst = l.pst; C.hdv = l.hdv; C.mhd = l.mhd; C.plan = l.plan; C.leg = l.leg;
    C.flags = l.flags; C.xs = l.xs; C.u0 = l.u0; C.sleg = l.sleg; C.u = l.u; C.foot = l.foot; C.x_pred = l.xp;
    C.status = l.st; C.iters = l.it; C.active = l.act;
    C.foot_traj = d_ft; C.x_traj = d_xt; C.hd_traj = d_hd; C.status_traj = d_stt; C.iters_traj = d_itt;
    C.steps_to_goal = d_sg;
    C.action_traj = d_act; C.vdes = l.vdes; C.pose0 = l.pose0;
    const double beta = std::sqrt(cf.g / cf.H), T = cf.dt, dt = T / f_cyc;
    {   // alip_des_vel(0.6, leg_ind) (MPC_LIP_modi.py:181-186)
        const double sh = std::sinh(beta * T), ch = std::cosh(beta * T);
        C.vdx = beta / std::tanh(T * beta / 2) * 0.6 * T / 2;
        C.vdy0 = (beta * sh) / (ch + 1);
    }
    C.ch_d = std::cosh(beta * dt); C.shb_d = std::sinh(beta * dt) / beta; C.bsh_d = std::sinh(beta * dt) * beta;
    C.td = dt / T;
    const unsigned g1 = (unsigned)((B + 255) / 256);
    hipLaunchKernelGGL(cl_init_kernel, dim3(g1), dim3(256), 0, st, C);
    HIPCHK(h, hipGetLastError());
    KP P = make_kp(h, B, true);
    P.goal = d_goal; P.cir = d_cir; P.nc = d_nc; P.elp = d_elp; P.ne = d_ne;
    P.x0 = l.xs; P.leg = l.sleg; P.u0 = l.u0; P.active = l.act;
    P.u_out = l.u; P.foot_out = l.foot; P.x_pred = l.xp; P.status = l.st; P.iters = l.it;
    // longest-first launch order of each tick (wave program; opt-in, ALIPMPC_CL_ORDER=1): it puts at most one long
    // instance on a SIMD, but a tick's time is set by its single slowest instance, a warm-started one whose line
    // search halves ~20 times per iteration (tools/cl_wstamps.py, profiles/r3/wst): 52.13 vs 52.00 ms per loop
    const char* oe = std::getenv("ALIPMPC_CL_ORDER");
    const bool order_ok = cf.program != ALIPMPC_PROGRAM_LANE && oe && std::strcmp(oe, "1") == 0;
    // Episode groups (ALIPMPC_CL_GROUPS, >= 256 episodes each): contiguous ranges of episodes whose ticks run on
    // streams of their own, so a tick that waits on one slow instance holds back only its group; the other groups'
    // launches fill the device meanwhile.  Every episode runs the same kernels on the same values (the kick is seeded
    // by the global episode index), so the outputs do not depend on the grouping (GPU test).
    int G = env_groups();
#ifdef ALIP_WSTAMP
    G = 1;   // (diagnostic records are indexed by the whole batch)
#endif
    if (order_ok) G = 1;   // (the opt-in launch order is a permutation of the whole batch)
    G = (int)std::max<long long>(1, std::min<long long>({(long long)G, (long long)Handle::MAXG, B / 256}));
    struct Grp {
        CLP C;
        KP P;
        hipStream_t s;
        unsigned g1;
    } grp[Handle::MAXG];
    const long long nn = n, SF = (long long)S * f_cyc;
    for (int g = 0; g < G; ++g) {
        const long long b0 = B * g / G, Bg = B * (g + 1) / G - b0;
        auto o = [&](auto& p, long long per) {
            if (p) p += b0 * per;
        };
        CLP c = C;
        c.B = Bg;
        c.b0 = b0;
        o(c.goal, 2); o(c.x, 5); o(c.pst, 2); o(c.hdv, 4); o(c.mhd, 3); o(c.plan, nn); o(c.leg, 1); o(c.flags, 1);
        o(c.xs, 5); o(c.u0, nn); o(c.sleg, 1); o(c.u, nn); o(c.foot, 3); o(c.x_pred, nn); o(c.status, 1);
        o(c.iters, 1); o(c.active, 1); o(c.foot_traj, 3LL * S); o(c.x_traj, 5LL * (S + 1)); o(c.hd_traj, 2LL * S);
        o(c.status_traj, SF); o(c.iters_traj, SF); o(c.steps_to_goal, 1); o(c.action_traj, 8 * SF); o(c.vdes, 2);
        o(c.pose0, 3);
        KP q = P;
        q.B = Bg;
        o(q.goal, 2); o(q.cir, 3LL * cf.nc_max); o(q.nc, 1); o(q.elp, 5LL * cf.ne_max); o(q.ne, 1); o(q.x0, 5);
        o(q.leg, 1); o(q.u0, nn); o(q.active, 1); o(q.u_out, nn); o(q.foot_out, 3); o(q.x_pred, nn); o(q.status, 1);
        o(q.iters, 1);
        grp[g].C = c;
        grp[g].P = q;
        grp[g].g1 = (unsigned)((Bg + 255) / 256);
        grp[g].s = st;
        if (G > 1) {
            if (!h->gst[g]) HIPCHK(h, hipStreamCreateWithFlags(&h->gst[g], hipStreamNonBlocking));
            if (!h->gev[g]) HIPCHK(h, hipEventCreateWithFlags(&h->gev[g], hipEventDisableTiming));
            grp[g].s = h->gst[g];
        }
    }
    if (G > 1 && !h->gev[Handle::MAXG]) HIPCHK(h, hipEventCreateWithFlags(&h->gev[Handle::MAXG], hipEventDisableTiming));
    const int ei = h->evi;
    h->evi = (ei + 1) % Handle::NEV;
    HIPCHK(h, hipEventRecord(h->ev[ei][0], st));
    if (G > 1) {   // fork
        HIPCHK(h, hipEventRecord(h->gev[Handle::MAXG], st));
        for (int g = 0; g < G; ++g) HIPCHK(h, hipStreamWaitEvent(grp[g].s, h->gev[Handle::MAXG], 0));
    }
    for (int s = 0; s < S; ++s) {
        for (int i = 0; i < f_cyc; ++i) {
            // rest_t = step_t - i * (step_t / f_cyc)   (main_sim_mpc.py:78)
            const double rest = T - i * (T / f_cyc);
            for (int g = 0; g < G; ++g) {
                CLP& Cg = grp[g].C;
                KP& Pg = grp[g].P;
                const hipStream_t sg = grp[g].s;
                Cg.s = s;
                Cg.i = i;
                Cg.ch_r = std::cosh(beta * rest); Cg.shb_r = std::sinh(beta * rest) / beta;
                Cg.bsh_r = std::sinh(beta * rest) * beta; Cg.tr = rest * (1.0 / T);
                hipLaunchKernelGGL(cl_project_kernel, dim3(grp[g].g1), dim3(256), 0, sg, Cg);
                HIPCHK(h, hipGetLastError());
                // wave program: after the first tick, solve last tick's long instances first (same bits per instance)
                Pg.order = nullptr;
                if (order_ok && (s > 0 || i > 0)) {
                    hipLaunchKernelGGL(cl_order_kernel, dim3(1), dim3(CL_ORDER_THREADS), 0, sg, (const int32_t*)l.it,
                                       (const uint8_t*)l.act, (long long)B, l.ord);
                    HIPCHK(h, hipGetLastError());
                    Pg.order = l.ord;
                }
                // each group's own counter pair (after the ring): its launches run in order on its stream, and no
                // other group or call can take the pair while one of them is in flight (ring pairs taken
                // per tick let a group running ticks ahead land on a pair another group's launch still used)
                Pg.queue = h->dq + 2 * (Handle::NQ + g);
#ifdef ALIP_WSTAMP
                {   // diagnostic record slots of this tick: (s f_cyc + i) B + instance
                    const long long base = ((long long)s * f_cyc + i) * B;
                    HIPCHK(h, hipMemcpyToSymbolAsync(HIP_SYMBOL(alip::g_wstamp_base), &base, sizeof(base), 0,
                                                     hipMemcpyHostToDevice, sg));
                    HIPCHK(h, hipStreamSynchronize(sg));   // &base is a stack value
                }
#endif
                HIPCHK(h, launch_solve(h, Pg, sg, h->cl_split_it, h->cl_split_tr));
                hipLaunchKernelGGL(cl_update_kernel, dim3(grp[g].g1), dim3(256), 0, sg, Cg);
                HIPCHK(h, hipGetLastError());
            }
        }
    }
    if (G > 1) {   // join
        for (int g = 0; g < G; ++g) {
            HIPCHK(h, hipEventRecord(h->gev[g], grp[g].s));
            HIPCHK(h, hipStreamWaitEvent(st, h->gev[g], 0));
        }
    }
    HIPCHK(h, hipEventRecord(h->ev[ei][1], st));
    h->evlast = ei;
    h->timed = true;
    if (host) {
        if (foot_traj) HIPCHK(h, hipMemcpyAsync(foot_traj, l.ft, Bz * Sz * 3 * 8, hipMemcpyDeviceToHost, st));
        if (x_traj) HIPCHK(h, hipMemcpyAsync(x_traj, l.xt, Bz * (Sz + 1) * 5 * 8, hipMemcpyDeviceToHost, st));
        if (hd_traj) HIPCHK(h, hipMemcpyAsync(hd_traj, l.hd, Bz * Sz * 2 * 8, hipMemcpyDeviceToHost, st));
        if (action_traj) HIPCHK(h, hipMemcpyAsync(action_traj, l.actd, Bz * Sz * Fz * 8 * 8, hipMemcpyDeviceToHost, st));
        if (status_traj) HIPCHK(h, hipMemcpyAsync(status_traj, l.stt, Bz * Sz * Fz * 4, hipMemcpyDeviceToHost, st));
        if (iters_traj) HIPCHK(h, hipMemcpyAsync(iters_traj, l.itt, Bz * Sz * Fz * 4, hipMemcpyDeviceToHost, st));
        if (steps_to_goal) HIPCHK(h, hipMemcpyAsync(steps_to_goal, l.sg, Bz * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
    }
    return ALIPMPC_OK;
}

int32_t alipmpc_trace_len(const alipmpc_cfg* cfg)
{
    if (!cfg || cfg->variant == ALIPMPC_VARIANT_DD || !(cfg->dt > 0)) return 0;
    // numpy arange length: ceil((stop - start) / step) with stop = dt + 0.01, step = 0.01; + the x_k row
    return 1 + (int32_t)std::ceil((cfg->dt + 0.01) / 0.01);
}

int alipmpc_trace_batch(void* handle, int64_t B, const double* x0, const double* u, double* trace, void* hip_stream)
{
    Handle* h = (Handle*)handle;
    if (!h) return ALIPMPC_EINVAL;
    const alipmpc_cfg& cf = h->cfg;
    if (cf.variant == ALIPMPC_VARIANT_DD) return fail(h, ALIPMPC_EUNSUPPORTED, "trace: LIP variants only");
    if (B < 0) return fail(h, ALIPMPC_EINVAL, "B < 0");
    if (B == 0) return ALIPMPC_OK;
    if (!x0 || !u || !trace) return fail(h, ALIPMPC_EINVAL, "missing pointer");
    HIPCHK(h, hipSetDevice(h->device));
    const int N = h->N, rows = alipmpc_trace_len(&cf);
    const size_t Bz = (size_t)B, nout = Bz * N * rows * 2;
    TrP T;
    std::memset(&T, 0, sizeof(T));
    T.B = B; T.N = N; T.rows = rows; T.step = 0.01;
    T.beta = std::sqrt(cf.g / cf.H);
    {
        const double b = T.beta, dT = cf.dt, ch = std::cosh(b * dT), sh = std::sinh(b * dT);
        const double A[25] = {ch, 0, sh / b, 0, 0, 0, ch, 0, sh / b, 0, sh * b, 0, ch, 0, 0,
                              0, sh * b, 0, ch, 0, 0, 0, 0, 0, 1};
        const double Bm[15] = {1 - ch, 0, 0, 0, 1 - ch, 0, -sh * b, 0, 0, 0, -sh * b, 0, 0, 0, 1};
        const double Dd = 5.0 * (ch - 1) * (ch - 1) + (sh * b) * (sh * b);
        const double Ch = -5.0 * (ch - 1) / Dd, Sh = -sh * b / Dd;
        const double W[15] = {Ch, 0, Sh, 0, 0, 0, Ch, 0, Sh, 0, 0, 0, 0, 0, 1};
        double BWA[25];
        std::memcpy(T.A, A, sizeof(A));
        std::memcpy(T.W, W, sizeof(W));
        mm(Bm, W, T.MB, 5, 3, 5);
        mm(T.MB, A, BWA, 5, 5, 5);
        for (int i = 0; i < 25; ++i) T.MA[i] = A[i] - BWA[i];
    }
    hipStream_t st = stream_of(h, hip_stream);
    const bool host = hip_stream == nullptr;
    if (host) {
        const size_t bytes = Bz * 5 * 8 + Bz * 5 * N * 8 + nout * 8 + 512;
        if (int rc = ensure_stage(h, bytes)) return rc;
        Carver cv{(char*)h->stage};
        double* dx = cv.take<double>(Bz * 5);
        double* du = cv.take<double>(Bz * 5 * N);
        double* dt_ = cv.take<double>(nout);
        HIPCHK(h, hipMemcpyAsync(dx, x0, Bz * 5 * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(du, u, Bz * 5 * N * 8, hipMemcpyHostToDevice, st));
        T.x0 = dx; T.u = du; T.trace = dt_;
    } else {
        T.x0 = x0; T.u = u; T.trace = trace;
    }
    const long long total = (long long)B * N * rows;
    hipLaunchKernelGGL(trace_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, T);
    HIPCHK(h, hipGetLastError());
    if (host) {
        HIPCHK(h, hipMemcpyAsync(trace, T.trace, nout * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
    }
    return ALIPMPC_OK;
}

int alipmpc_nominal_gait_batch(void* handle, int64_t B, double vx_max, const double* x, const int8_t* leg,
                               const double* vel_des_in, double* vel_des, double* foot, void* hip_stream)
{
    Handle* h = (Handle*)handle;
    if (!h) return ALIPMPC_EINVAL;
    const alipmpc_cfg& cf = h->cfg;
    if (cf.variant == ALIPMPC_VARIANT_DD) return fail(h, ALIPMPC_EUNSUPPORTED, "nominal gait: LIP variants only");
    if (B < 0) return fail(h, ALIPMPC_EINVAL, "B < 0");
    if (B == 0) return ALIPMPC_OK;
    if (!x || !foot || (!leg && !vel_des_in)) return fail(h, ALIPMPC_EINVAL, "missing pointer");
    HIPCHK(h, hipSetDevice(h->device));
    const size_t Bz = (size_t)B;
    NgP Q;
    std::memset(&Q, 0, sizeof(Q));
    Q.B = B;
    {
        const double b = std::sqrt(cf.g / cf.H), T = cf.dt, sh = std::sinh(b * T), ch = std::cosh(b * T);
        const double sigma = b / std::tanh(T * b / 2);   // beta coth(beta T / 2)
        Q.vdx = sigma * vx_max * T / 2;
        Q.vdy0 = (b * sh) / (ch + 1);
        Q.bsh = sh * b;
        Q.ch = ch;
        Q.ibv = 1.0 / (-sh * b);
    }
    hipStream_t st = stream_of(h, hip_stream);
    const bool host = hip_stream == nullptr;
    if (host) {
        if (int rc = ensure_stage(h, Bz * 8 * (5 + 2 + 2 + 2) + Bz + 5 * 256)) return rc;   // 5 carves, 256 B aligned
        Carver cv{(char*)h->stage};
        double* dx = cv.take<double>(Bz * 5);
        double* dvi = cv.take<double>(Bz * 2);
        double* dvo = cv.take<double>(Bz * 2);
        double* df = cv.take<double>(Bz * 2);
        int8_t* dl = cv.take<int8_t>(Bz);
        HIPCHK(h, hipMemcpyAsync(dx, x, Bz * 5 * 8, hipMemcpyHostToDevice, st));
        if (vel_des_in) HIPCHK(h, hipMemcpyAsync(dvi, vel_des_in, Bz * 2 * 8, hipMemcpyHostToDevice, st));
        if (leg) HIPCHK(h, hipMemcpyAsync(dl, leg, Bz, hipMemcpyHostToDevice, st));
        Q.x = dx; Q.vin = vel_des_in ? dvi : nullptr; Q.leg = leg ? dl : nullptr;
        Q.vout = vel_des ? dvo : nullptr; Q.foot = df;
    } else {
        Q.x = x; Q.vin = vel_des_in; Q.leg = leg; Q.vout = vel_des; Q.foot = foot;
    }
    hipLaunchKernelGGL(nominal_gait_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, Q);
    HIPCHK(h, hipGetLastError());
    if (host) {
        if (vel_des) HIPCHK(h, hipMemcpyAsync(vel_des, Q.vout, Bz * 2 * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipMemcpyAsync(foot, Q.foot, Bz * 2 * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
    }
    return ALIPMPC_OK;
}

#ifdef ALIP_STAMPS
int alipmpc_dbg_stamps(unsigned long long* out, int reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(alip::g_stamps), sizeof(unsigned long long) * alip::NSTAMP) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[alip::NSTAMP] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(alip::g_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return alip::NSTAMP;
}
#endif

#ifdef ALIP_WSTAMP
// diagnostic: copy the first `slots` per-instance records (8 values each) of the wave program and reset the base
int alipmpc_dbg_wstamps(unsigned long long* out, long long slots)
{
    if (slots > alip::WSTAMP_CAP) slots = alip::WSTAMP_CAP;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(alip::g_wstamp), sizeof(unsigned long long) * 8 * (size_t)slots) != hipSuccess)
        return -1;
    const long long z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(alip::g_wstamp_base), &z, sizeof(z)) != hipSuccess) return -1;
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(alip::g_wstamp)) != hipSuccess ||
        hipMemset(p, 0, sizeof(unsigned long long) * 8 * (size_t)alip::WSTAMP_CAP) != hipSuccess)
        return -1;
    return (int)slots;
}
#endif

const char* alipmpc_build_id(void)
{
#ifdef ALIP_BUILD_ID
    return ALIP_BUILD_ID;
#else
    return "unknown";
#endif
}

double alipmpc_last_kernel_ms(void* handle)
{
    Handle* h = (Handle*)handle;
    if (!h || !h->timed) return 0.0;
    if (h->evlast < 0) return 0.0;
    hipEvent_t e0 = h->ev[h->evlast][0], e1 = h->ev[h->evlast][1];
    if (hipEventSynchronize(e1) != hipSuccess) return 0.0;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e0, e1) != hipSuccess) return 0.0;
    return (double)ms;
}

const char* alipmpc_last_error(void* handle)
{
    Handle* h = (Handle*)handle;
    return h ? h->err.c_str() : "null handle";
}

int alipmpc_solve_slots(void* handle, int64_t* slots)
{
    Handle* h = (Handle*)handle;
    if (!h || !slots) return fail(h, ALIPMPC_EINVAL, "null argument");
    HIPCHK(h, hipSetDevice(h->device));
    unsigned res = 0;
    KP P = make_kp(h, 1, true);
    HIPCHK(h, launch(h, true, P, h->own, &res));
    if (h->lane_nct >= 0)
        *slots = (int64_t)res * (h->cfg.precision == ALIPMPC_PREC_FP32 ? lane::lanes_of<float>() : lane::lanes_of<double>());
    else
        *slots = (int64_t)res * WAVES_PER_BLOCK;
    return ALIPMPC_OK;
}

int alipmpc_lane_handoffs(void* handle, void* hip_stream, int64_t* count)
{
    Handle* h = (Handle*)handle;
    if (!h || !count) return fail(h, ALIPMPC_EINVAL, "null argument");
    *count = 0;
    hipStream_t st = stream_of(h, hip_stream);
    void* p = nullptr;
    {
        std::lock_guard<std::mutex> lk(h->split_mtx);
        auto it = h->redo.find(st);
        if (it != h->redo.end()) p = it->second.p;
    }
    if (!p) return ALIPMPC_OK;
    uint32_t c = 0;
    if (hipStreamSynchronize(st) != hipSuccess || hipMemcpy(&c, p, sizeof(c), hipMemcpyDeviceToHost) != hipSuccess)
        return fail(h, ALIPMPC_EHIP, "alipmpc_lane_handoffs: reading the hand-off count");
    *count = c;
    return ALIPMPC_OK;
}

int alipmpc_solve_launches(void* handle, int64_t B, int32_t* launches, int32_t* team)
{
    Handle* h = (Handle*)handle;
    if (!h || !launches || !team) return fail(h, ALIPMPC_EINVAL, "null argument");
    int64_t slots = 0;
    if (int rc = alipmpc_solve_slots(handle, &slots)) return rc;
    // launch_solve's conditions for the split form (no order / active mask on the batch API)
    const bool split = split_form(h, B, h->split_it, h->split_tr, slots);
    *launches = split ? 2 : 1;
    *team = split && h->split_tr > 0 && h->cfg.precision != ALIPMPC_PREC_FP32 ? TEAM_WAVES : 1;
    return ALIPMPC_OK;
}

const char* alipmpc_solve_program(void* handle)
{
    Handle* h = (Handle*)handle;
    if (!h) return "";
    static thread_local char buf[96];
    const alipmpc_cfg& c = h->cfg;
    const char* r = c.precision == ALIPMPC_PREC_FP32 ? "float" : "double";
    if (c.variant == ALIPMPC_VARIANT_DD) {
        const int rpl = h->mo4 / WAVE;
        std::snprintf(buf, sizeof(buf), "dd_solve_kernel<%d,%d>", h->N, rpl);
    } else if (h->lane_nct >= 0) {
        std::snprintf(buf, sizeof(buf), "lane_kernel<%d,%d,%s,%s>", h->N, h->lane_nct,
                      c.variant == ALIPMPC_VARIANT_MODI ? "true" : "false", r);
    } else {
        std::snprintf(buf, sizeof(buf), "solve_kernel<%d,%d,%s>", h->N, h->mo4 / 4, r);
    }
    return buf;
}

void alipmpc_destroy(void* handle)
{
    Handle* h = (Handle*)handle;
    if (!h) return;
    hipSetDevice(h->device);
    if (h->own) hipStreamSynchronize(h->own);
    for (double* d : {h->dGp, h->dEp, h->dGu, h->dEu})
        if (d) (void)hipFree(d);
    if (h->dq) hipFree(h->dq);
    if (h->dlk) hipFree(h->dlk);
    if (h->dlkf) hipFree(h->dlkf);
    if (h->stage) hipFree(h->stage);
    if (h->rstage) hipFree(h->rstage);
    for (auto& kv : h->split)
        if (kv.second.p) hipFree(kv.second.p);
    for (auto& kv : h->redo)
        if (kv.second.p) hipFree(kv.second.p);
    for (auto& pr : h->ev)
        for (hipEvent_t e : pr)
            if (e) hipEventDestroy(e);
    if (h->own) hipStreamDestroy(h->own);
    for (int g = 0; g < Handle::MAXG; ++g) {
        if (h->gst[g]) hipStreamDestroy(h->gst[g]);
        if (h->gev[g]) hipEventDestroy(h->gev[g]);
    }
    if (h->gev[Handle::MAXG]) hipEventDestroy(h->gev[Handle::MAXG]);
    delete h;
}

}  // extern "C"
#endif  // ALIP_PART_HOST
