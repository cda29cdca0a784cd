/*
 * alipmpc.h — C ABI of the MI355X batched ALIP-MPC-CBF footstep planner (libalipmpc.so).
 *
 * Drop-in boundary for the reference's per-step NLP solve.  The reference has no C ABI: its planner API
 * is the Python class MPCCBF (MPC_LIP_modi.py:13-391) whose solveMPCCBF (MPC_LIP_modi.py:197-301)
 * hands an NLP plugin object LIP_Prob (MPC_LIP_modi.py:394-655: objective / gradient / constraints /
 * jacobian) to cyipopt.Problem + nlp.solve(u0) (MPC_LIP_modi.py:274-296).  Each entry point below
 * replaces one of those interfaces for a whole batch of independent instances:
 *
 *   alipmpc_solve_batch  <- MPCCBF.select_obs + MPCCBF.solveMPCCBF + cyipopt.Problem.solve, and the
 *                           rollout of MPCCBF.gen_control_test   (MPC_LIP_modi.py:90-112,197-301,325-338;
 *                           MPC_LIP_sig_step.py:89-111,184-278; MPC_DD_sig_step.py:70-97,123-193)
 *   alipmpc_eval_batch   <- LIP_Prob.objective/gradient/constraints/jacobian + the cl/cu/goal set-up
 *                           of solveMPCCBF                     (MPC_LIP_modi.py:205-271,430-583;
 *                           MPC_LIP_sig_step.py:195-254,372-496; MPC_DD_sig_step.py:127-141,351-477)
 *   alipmpc_default_cfg  <- the hard-coded constants of MPCCBF.__init__ / LIP_Prob.__init__
 *                           (MPC_LIP_modi.py:17-45,397-411; MPC_LIP_sig_step.py:17-44,340-353;
 *                           MPC_DD_sig_step.py:15-40,323-338)
 *
 * Conventions
 *   - The caller owns every buffer.  hip_stream == NULL: all pointers are HOST pointers; the library
 *     stages them through its own device workspace and synchronises before returning.
 *     hip_stream != NULL: all pointers are DEVICE pointers (hipMalloc / torch CUDA tensors) and the call
 *     is asynchronous on that stream (no host synchronisation; graph-capturable).  The only device allocation
 *     is the split launch's record buffer (alipmpc_solve_launches): one per stream, made by the stream's first
 *     split solve, sized for the resident slots and kept until alipmpc_destroy — a capture on a stream that has
 *     none yet records the one-phase form.  A captured graph uses its capture stream's buffer: replay it on that
 *     stream (or ordered with the solves there).  At most 8 streams per handle hold one (kept until destroy, never
 *     evicted); solves on a further stream run the one-phase form (same bits).  ALIPMPC_STREAM_NULL selects device pointers on
 *     the null (default) stream, whose handle value is 0.
 *   - Every LIP solve launch takes one of the handle's 64 work-queue counter pairs (a ring; each pair is
 *     reset by the last wave of the launch that used it).  A solve captured into a hipGraph bakes in one
 *     pair: do not replay such a graph concurrently with itself, and keep fewer than 64 solve launches of
 *     one handle in flight at once (across all streams), or two launches share counters and instances
 *     are skipped or solved twice.  alipmpc_closed_loop_batch's ticks do not take ring pairs: each of its
 *     episode groups owns one pair of its own (its launches run in order on the group's stream).
 *   - Row-major, instance-major arrays ("B x k" = k contiguous values per instance).
 *   - Return 0 on success, a negative ALIPMPC_E* code on error; alipmpc_last_error(h) gives the text.
 *   - There is no CPU execution path: a handle needs a visible gfx950 device.
 *   - One handle per host thread / stream; distinct handles are independent.
 *
 * Problem layout (variant 0 = "modi" MPC_LIP_modi.py, 1 = "sig_step" MPC_LIP_sig_step.py, 2 = "dd"
 * MPC_DD_sig_step.py):
 *   LIP (0,1): state x = [px, py, vx, vy, theta] (sdim = 5), decision u = [u_1..u_N], u_i in R^5
 *              (n = 5N), foothold p_i = W(u_i - A x_i) = [foot x, foot y, turn].
 *   DD  (2):   state x = [px, py, theta] (sdim = 3), decision u = [v_1, w_1, ..., v_N, w_N] (n = 2N).
 *   Constraint rows are laid out in a FIXED padded order, rows_per_step rows per step k = 0..N-1:
 *     LIP: [vbx, vby, circle slot 0..nc_max-1, ellipse slot 0..ne_max-1, leg, dtheta, (f_en if modi)]
 *     DD : [circle slot 0..nc_max-1, ellipse slot 0..ne_max-1, f_en]
 *   select_obs (modi) compacts the kept obstacles, in input order, into the first slots; unused slots
 *   are inactive (row_active = 0, cl = -inf, cu = +inf, value/Jacobian rows = 0).  Dropping the
 *   inactive rows gives exactly the reference's row order.
 */
#ifndef ALIPMPC_H
#define ALIPMPC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ALIPMPC_VARIANT_MODI 0
#define ALIPMPC_VARIANT_SIG_STEP 1
#define ALIPMPC_VARIANT_DD 2

#define ALIPMPC_PREC_FP64 0
#define ALIPMPC_PREC_FP32 1

/* IPOPT-compatible status codes written to status[] (cyipopt info['status']) */
#define ALIPMPC_SOLVE_SUCCEEDED 0
#define ALIPMPC_SOLVED_TO_ACCEPTABLE_LEVEL 1
#define ALIPMPC_INFEASIBLE_PROBLEM_DETECTED 2
#define ALIPMPC_MAXIMUM_ITERATIONS_EXCEEDED (-1)
#define ALIPMPC_ERROR_IN_STEP_COMPUTATION (-3)   /* KKT regularisation exhausted; last iterate returned */
#define ALIPMPC_INVALID_NUMBER_DETECTED (-13)    /* cfg.goal_singular = ABORT only: see alipmpc_cfg */
/* rollout only: the instance had already reached its goal, no solve was run at this step */
#define ALIPMPC_ROLLOUT_DONE (-10)

/* error codes */
#define ALIPMPC_OK 0
#define ALIPMPC_EINVAL (-1)
#define ALIPMPC_ENODEV (-2)
#define ALIPMPC_EHIP (-3)
#define ALIPMPC_EUNSUPPORTED (-4)

/* cfg.program */
#define ALIPMPC_PROGRAM_WAVE 0
#define ALIPMPC_PROGRAM_LANE 1

/* hip_stream value meaning "device pointers, asynchronous on the null (default) stream" */
#define ALIPMPC_STREAM_NULL ((void*)(intptr_t)-1)

#define ALIPMPC_MAX_N 6      /* horizon limit of the kernels (n = 5N <= 32 -> two 16-column MFMA tiles) */
#define ALIPMPC_MAX_OBS 24   /* nc_max + ne_max limit (and N * rows_per_step <= 128) */

typedef struct alipmpc_cfg {
    int32_t N;          /* horizon (reference: step = 3) */
    int32_t nc_max;     /* circle slots per instance (raw count before select_obs) */
    int32_t ne_max;     /* ellipse slots per instance */
    int32_t variant;    /* ALIPMPC_VARIANT_* */
    int32_t max_iter;   /* interior-point iteration cap */
    int32_t precision;  /* ALIPMPC_PREC_FP64 / _FP32 (device arithmetic; host buffers stay fp64).  With
                           FP32 and tol / acceptable_tol still at the fp64 defaults (1e-8 / 1e-6, below
                           fp32 resolution), alipmpc_create uses the fp32 defaults: 1e-4 / 1e-3 for
                           N <= 3, 3e-4 / 3e-3 for N > 3 */
    int32_t select_obs; /* 1: MPCCBF.select_obs range filter (modi) */
    int32_t detour;     /* 1: local-goal detour heuristic of solveMPCCBF (modi, sig_step) */
    double tol;         /* overall KKT tolerance (IPOPT tol, default 1e-8) */
    double acceptable_tol;
    double dt, H, g;    /* step period T, LIP height, gravity */
    double leg2_max;    /* leg length^2 bound */
    double bvx_lo, bvx_hi, bvy_lo, bvy_hi; /* body-frame velocity bounds (DD: v bounds in bvx_*) */
    double dtheta_max;  /* turning bound (DD: omega bound) */
    double q, p, r;     /* cost weights: position, first-step position, heading */
    double gamma;       /* D-CBF decay */
    double s;           /* f_en turning weight */
    double detect_r2;   /* select_obs range^2 */
    double dd_t;        /* DD control-smoothness weight */
    double mu_init;     /* initial barrier parameter */
    int32_t program;    /* device program (no reference counterpart; the arithmetic of the interior point is the
                           same in both): ALIPMPC_PROGRAM_WAVE — one instance per wavefront (solve_kernel,
                           latency-optimised: small batches); ALIPMPC_PROGRAM_LANE — one instance per lane
                           (lane_kernel, throughput-optimised: batches of 10^5+ instances; N = 3 with circles only,
                           modi / sig_step, otherwise alipmpc_create returns ALIPMPC_EUNSUPPORTED).  A per-handle
                           choice, never a function of B: an instance's result does not depend on its batch. */
    int32_t goal_singular; /* a planned state exactly on the goal, where the target heading atan2(g - p) has 0 / 0
                           derivatives (the reference's cal_dtar_ang_du, MPC_LIP_modi.py:650-655, returns NaN there):
                           ALIPMPC_GOAL_SINGULAR_ZERO (0, default) — take them as 0 (atan2(0, 0) = 0 held locally
                           constant; a deviation); ALIPMPC_GOAL_SINGULAR_ABORT (1) — the
                           reference's path: IPOPT's gradient check (Eval_Error on a non-finite objective gradient)
                           ends the solve with status ALIPMPC_INVALID_NUMBER_DETECTED (-13) at the first iterate
                           (starting point or accepted step) with such a state, and that iterate is returned.
                           (Fills the struct's tail padding: sizeof(alipmpc_cfg) is unchanged.) */
    int32_t restoration;   /* what follows a failed filter line search (IPOPT's default path; no reference option
                           selects it): ALIPMPC_RESTORATION_IPOPT (0, default) — IPOPT's feasibility restoration phase:
                           the l1 feasibility problem min rho sum(p + n) + zeta/2 |D_R (x - x_R)|^2 s.t. c(x) - s - p + n
                           = 0 (rho = 1000, zeta = sqrt(mu)) solved by the same interior point until an iterate the
                           original filter accepts with 0.9 of the violation, status 2 (Infeasible_Problem_Detected)
                           only when it converges to a point of local infeasibility;
                           ALIPMPC_RESTORATION_SUBSTITUTE (1) — the rounds-1..5 substitute: the shortest trial step,
                           slacks reset onto c(u), filter reset, status 2 after 6 such events.  The DD variant always
                           runs the substitute.  fp64 wave program: split launches run the phase in their second
                           launch (a failed search in the first cuts the instance there).  Lane program (both
                           precisions) and fp32 wave program: an instance whose search fails is handed to the fp64
                           wave program, which solves it from its start (alipmpc_lane_handoffs counts them); the fp64
                           workspace must then fit the LDS too (alipmpc_create: ALIPMPC_EUNSUPPORTED otherwise). */
    int32_t reserved_;  /* zero */
} alipmpc_cfg;

#define ALIPMPC_GOAL_SINGULAR_ZERO 0
#define ALIPMPC_GOAL_SINGULAR_ABORT 1

#define ALIPMPC_RESTORATION_IPOPT 0
#define ALIPMPC_RESTORATION_SUBSTITUTE 1

/* Fill *out with the reference's constants for a variant and horizon.  nc_max = ne_max = 6, precision
 * fp64, max_iter = the reference's IPOPT cap (modi 30, sig_step 20, DD 40). */
int alipmpc_default_cfg(int32_t variant, int32_t N, alipmpc_cfg* out);

/* Rows per step and total padded rows (m_max) of the fixed constraint layout for cfg. */
int32_t alipmpc_rows_per_step(const alipmpc_cfg* cfg);
int32_t alipmpc_num_vars(const alipmpc_cfg* cfg);

/* device: HIP device ordinal (>= 0).  Returns ALIPMPC_ENODEV when no gfx950 device is visible. */
int alipmpc_create(const alipmpc_cfg* cfg, int device, void** handle);

/*
 * Solve B independent NLP instances.
 *   x0    B x sdim         initial state (MPCCBF.gen_control_test `state`)
 *   goal  B x 2            goal position (MPCCBF `goals`)
 *   leg   B                od_ev = +-1 (the reference passes -leg_ind)
 *   cir   B x nc_max x 3   inflated circles [cx, cy, r]   (cir_cbf); nc[b] of them valid
 *   elp   B x ne_max x 5   inflated ellipses [cx, cy, a, b, phi] (elp_cbf); ne[b] valid (may be NULL if ne_max == 0)
 *   u0    B x n            initial guess (init_guess)
 *   last_u B x 2           DD only: previous control (may be NULL otherwise)
 * Outputs (any output pointer may be NULL except u_out):
 *   u_out    B x n         solution u
 *   foot_out B x 3         p_list[0] = W(u_1 - A x0) (LIP) / first control [v, w, 0] (DD)
 *   x_pred   B x N x sdim  predicted states x_1..x_N (xk_list[1:])
 *   status   B             IPOPT-compatible status
 *   iters    B             interior-point iterations used
 */
int alipmpc_solve_batch(void* handle, int64_t B,
                        const double* x0, const double* goal, const int8_t* leg,
                        const double* cir, const int32_t* nc,
                        const double* elp, const int32_t* ne,
                        const double* u0, const double* last_u,
                        double* u_out, double* foot_out, double* x_pred,
                        int32_t* status, int32_t* iters,
                        void* hip_stream);

/*
 * Evaluate the NLP callbacks and the set-up at given u (parity / oracle hook).  m_max = N*rows_per_step.
 *   f B, grad B x n, c B x m_max, J B x m_max x n, cl/cu B x m_max, goal_eff B x 2 (after detour),
 *   row_active B x m_max.  Any output may be NULL.
 *   Kernels: N = 3 with circle slots only runs the sweep kernel (lane-per-instance set-up, wave-cooperative
 *   J stores), every other shape eval_kernel; both give the same bits.  Dev knobs (environment):
 *   ALIPMPC_EVAL_KERNEL=group (read by alipmpc_create) forces eval_kernel, ALIPMPC_SWEEP_SHAPE=641 (read per
 *   call) the 64-instance sweep shape.
 */
int alipmpc_eval_batch(void* handle, int64_t B,
                       const double* x0, const double* goal, const int8_t* leg,
                       const double* cir, const int32_t* nc,
                       const double* elp, const int32_t* ne,
                       const double* u, const double* last_u,
                       double* f, double* grad, double* c, double* J,
                       double* cl, double* cu, double* goal_eff, int8_t* row_active,
                       void* hip_stream);

/*
 * Closed-loop receding-horizon rollout of B independent episodes for up to S steps on an ideal ALIP plant
 * (the batch harness that replaces the data_log replay loop: main_sim_mpc.py:66-131 driving
 * logger_mpc.py:318-341 gen_nex_foot_input -> MPCCBF.gen_control_test).  Step t: solve every active
 * instance (as alipmpc_solve_batch), execute the first planned step (x <- x_pred[0], the state at the next
 * touchdown = get_next_states over a full step), switch stance (leg <- -leg), warm-start the next solve
 * from the plan (modi: previous x_mpc_tar unshifted, logger_mpc.py:325-331; sig_step: [g2..gN, gN],
 * MPC_LIP_sig_step.py:186-189; DD: previous controls and last_u <- first control), and retire the
 * instance once close_2_goal holds (the episode stops after that step, main_sim_mpc.py:121-131).
 * Inputs as alipmpc_solve_batch (x0/leg/u0/last_u = the first step's).  Outputs (any may be NULL):
 *   foot_traj     B x S x 3        p_list[0] of each step (NaN after the goal)
 *   x_traj        B x (S+1) x sdim touchdown states x^(0) = x0, x^(1), ...
 *   status_traj   B x S            solve status per step (ALIPMPC_ROLLOUT_DONE after the goal)
 *   iters_traj    B x S            interior-point iterations per step
 *   steps_to_goal B                steps taken until close_2_goal (-1: not within S)
 *   u_traj        B x S x n        the plan (solution u) of every step (NaN after the goal); with x_traj it
 *                                  feeds alipmpc_trace_batch for the per-step predicted traces
 * Host pointers when hip_stream == NULL, else device pointers (asynchronous; S solve launches + S small
 * plant-update launches on the stream, no host synchronisation).
 */
int alipmpc_rollout_batch(void* handle, int64_t B, int32_t S,
                          const double* x0, const double* goal, const int8_t* leg,
                          const double* cir, const int32_t* nc,
                          const double* elp, const int32_t* ne,
                          const double* u0, const double* last_u,
                          double* foot_traj, double* x_traj, int32_t* status_traj, int32_t* iters_traj,
                          int32_t* steps_to_goal, double* u_traj, void* hip_stream);

/*
 * Closed loop at the reference's control rate: B episodes of up to S walking steps with f_cyc MPC solves per
 * step (main_sim_mpc.py:41,65-135, f_cyc = 40: one solve per 10 ms tick of a 0.4 s step) on an ALIP plant —
 * the batch harness of Logger.set_stf_head / gen_nex_foot_input (data_procs/logger_mpc.py:270-371).
 * Tick i of step s (rest_t = T - i T / f_cyc, main_sim_mpc.py:78):
 *   i == 0: set_stf_head with the plant heading: nex_turn <- tube_func(nex_turn, hd), hd_input_pr <- avg_hd(hd),
 *           hd_input_cos <- hd (logger_mpc.py:208-215, 270-300; nex_turn = 0 and mpc_hds_list = the initial heading
 *           initially — the Logger's 0 in its robot frame, whose origin is the initial pose, logger_mpc.py:27,90);
 *   x_nex = get_next_states(pos, vel, hd, [stance foot, hd_input_pr], rest_t) (MPC_LIP_modi.py:149-178);
 *   solve at x_nex with od_ev = -leg_ind; warm start [x_nex] x 3 on the episode's first solve, then the
 *   previous plan x_mpc_tar (logger_mpc.py:327-333 with the driver's num_step >= 1; sig_step: [g2..gN, gN]);
 *   nex_turn <- p_list[0][2], mpc_hds_list <- hd_list;
 *   the plant moves dt = T / f_cyc around the stance foot with the heading advancing hd_input_pr dt / T (the
 *   model get_next_states assumes), plus a velocity kick kick * U(-1, 1) per axis from splitmix64(seed,
 *   episode, step, tick, axis) (plant mismatch; kick = 0: the ideal plant);
 *   after the last tick: touchdown — the stance foot becomes p_list[0][0:2] of that solve, leg_ind <- -leg_ind;
 *   the episode stops there if any earlier solve reported close_2_goal (the driver checks real_close at the
 *   foot change before updating it, main_sim_mpc.py:106-135).
 * Inputs: x0 B x 5 plant state at the first touchdown, foot0 B x 2 its stance foot, goal B x 2, leg B leg_ind
 * (the reference starts at -1), obstacles as alipmpc_solve_batch.  Outputs (any may be NULL):
 *   foot_traj B x S x 3 (p_list[0] of each step's last solve, NaN after the stop), x_traj B x (S+1) x 5
 *   (touchdown states), hd_traj B x S x 2 (hd_input_pr, hd_input_cos of each step), status_traj / iters_traj
 *   B x S x f_cyc (ALIPMPC_ROLLOUT_DONE after the stop), steps_to_goal B (-1: not within S), action_traj
 *   B x S x f_cyc x 8: the task-space-controller command of every tick (Logger.gen_nex_foot_input +
 *   gen_tsc_control, logger_mpc.py:318-384: [foot_input x, y, 0, hd_input_pr / f_cyc (i + 4.5) + hd_input_cos,
 *   nex_pos_fot_loc x, y, nex_vel_fot_loc x, 0] in the Logger's robot-global frame = the map frame moved to the
 *   initial pose; vel_des starts at alip_des_vel(0.6, leg_ind) and follows mpc_state_tar as main_sim_mpc.py:54,
 *   88, 112 do; NaN after the stop).
 * LIP variants only (DD: ALIPMPC_EUNSUPPORTED).  Host / device pointers as alipmpc_solve_batch; S * f_cyc solve
 * launches plus two small kernels per tick on the stream.
 */
int alipmpc_closed_loop_batch(void* handle, int64_t B, int32_t S, int32_t f_cyc, double kick, uint64_t seed,
                              const double* x0, const double* foot0, const double* goal, const int8_t* leg,
                              const double* cir, const int32_t* nc, const double* elp, const int32_t* ne,
                              double* foot_traj, double* x_traj, double* hd_traj, int32_t* status_traj,
                              int32_t* iters_traj, int32_t* steps_to_goal, double* action_traj, void* hip_stream);

/* Nominal gait of a batch (replaces MPCCBF.alip_des_vel / cal_foot_with_veldes, MPC_LIP_modi.py:181-194, used by
 * the driver at main_sim_mpc.py:54 and the ALIP-only loggers):
 *   vel_des = alip_des_vel(vx_max, leg_ind) = [sigma vx_max T / 2, 0.5 (-0.5 leg_ind step_gap) beta sinh(beta T) /
 *             (cosh(beta T) + 1)], sigma = beta coth(beta T / 2), step_gap = 0.3 — or the given vel_des_in (B x 2),
 *   foot    = cal_foot_with_veldes(x, vel_des) = B_vel^-1 (vel_des - (A x)[2:4]), B_vel = B[2:4, 0:2].
 * x B x 5 states, leg B leg_ind (ignored when vel_des_in is given), vel_des B x 2 (may be NULL), foot B x 2.
 * Host pointers with hip_stream = NULL (synchronous), device pointers otherwise. */
int alipmpc_nominal_gait_batch(void* handle, int64_t B, double vx_max, const double* x, const int8_t* leg,
                               const double* vel_des_in, double* vel_des, double* foot, void* hip_stream);

/* Rows per planned step of alipmpc_trace_batch: 1 + len(np.arange(0, dt + 0.01, 0.01)) (42 at dt = 0.4);
 * 0 for the DD variant. */
int32_t alipmpc_trace_len(const alipmpc_cfg* cfg);

/*
 * Dense CoM traces of plans — the pos_det output of MPCCBF.gen_control_test (MPC_LIP_modi.py:117-122) built
 * by MPCCBF.xk_track_det (MPC_LIP_modi.py:304-322), i.e. the 126 x 2 rows per plan of the reference's
 * data_log *_pred_full_end.pkl at N = 3 (main_sim_mpc.py:117, logger_mpc.py:473).  For each instance and
 * step k = 0..N-1: row 0 = x_k[0:2], then the ALIP flow from x_k around the stance foot p_k at t = 0, 0.01,
 * ..., with x_{k+1} = M_A x_k + M_B u_k and p_k = W(u_k - A x_k) as gen_control_test forms them.
 *   x0 B x 5, u B x 5N (a solve's u_out)  ->  trace B x N x alipmpc_trace_len(cfg) x 2.
 * LIP variants only (DD: ALIPMPC_EUNSUPPORTED).  Host / device pointers as alipmpc_solve_batch.
 */
int alipmpc_trace_batch(void* handle, int64_t B, const double* x0, const double* u, double* trace,
                        void* hip_stream);

/* Instances this handle's solve kernel holds resident on its device at once (solve_kernel: resident
 * workgroups x 4 waves, one instance per wave; lane_kernel: resident waves x instances per wave).  A wave-program
 * batch that fits these slots launches one wave per instance (as a split launch, see alipmpc_solve_launches); a
 * larger one — and every lane-program batch — runs as a persistent grid of the resident workgroups whose waves
 * (lanes) pull instances from a per-launch work queue.  Every form runs the same per-instance arithmetic, so an
 * instance's result does not depend on B (a batch solved whole or in chunks is bit-identical).  0 for the DD
 * variant (always one wave per instance).  No reference counterpart (scheduling of the batched replacement). */
int alipmpc_solve_slots(void* handle, int64_t* slots);

/* Kernel launches one alipmpc_solve_batch of B instances runs on this handle: 2 for a split launch (wave program,
 * 2 <= B <= alipmpc_solve_slots, and ALIPMPC_SPLIT_IT > 0 — phase 1 up to that many iterations, phase 2 resumes the
 * unfinished instances from their exact loop-state records — or, fp64, ALIPMPC_SPLIT_TR > 0), 1 otherwise; *team = the
 * team size (4 waves) when phase 1 also cuts instances by their line-search trial count (ALIPMPC_SPLIT_TR > 0, fp64
 * only) into team records that phase 2 runs on a team each, else 1.
 * It reports the form of an eager launch on a stream that holds, or can still get, a record buffer: a launch
 * captured into a graph on a stream without one, or on a ninth stream, runs the one-phase form (1 launch).
 * Profiling tools use it to turn per-dispatch figures into per-solve ones.  No reference counterpart. */
int alipmpc_solve_launches(void* handle, int64_t B, int32_t* launches, int32_t* team);

/* Lane program (either precision) or fp32 wave program with cfg.restoration = ALIPMPC_RESTORATION_IPOPT: the instances
 * of the last solve on this stream whose line search failed in that program and which were therefore solved, from
 * their start, by the fp64 wave program's restoration-capable work queue (IPOPT's restoration phase: DESIGN.md §2
 * item 4).  Synchronises the stream.  0 for other programs / restoration modes.  No reference counterpart. */
int alipmpc_lane_handoffs(void* handle, void* hip_stream, int64_t* count);

/* The device program this handle's solves run (cfg.program): "solve_kernel<N,rows/4,type>" (one instance per
 * wavefront; launched as one wave per instance when the batch fits alipmpc_solve_slots, as the persistent
 * work queue otherwise — the same bits per instance either way), "lane_kernel<N,circle slots,modi,type>" (one
 * instance per lane) or "dd_solve_kernel<N,row groups>".  No reference counterpart.  The string is owned by
 * the library. */
const char* alipmpc_solve_program(void* handle);

/* Duration in milliseconds of the most recent solve kernel launch on this handle, measured with HIP
 * events on the launch stream (0 if none). */
double alipmpc_last_kernel_ms(void* handle);

/* Identifier of this library build: 16 hex digits of a sha256 over the sources and compile flags it was built from
 * (alipmpc/build.py).  Profiles and counter records carry it, so tools never attach one build's counters to another
 * build's measurement.  No reference counterpart. */
const char* alipmpc_build_id(void);

const char* alipmpc_last_error(void* handle);
void alipmpc_destroy(void* handle);

#ifdef __cplusplus
}
#endif
#endif /* ALIPMPC_H */
