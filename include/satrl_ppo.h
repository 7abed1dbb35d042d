/*
 * satrl_ppo.h -- C ABI of the fused PPO minibatch-step kernels (gfx950).
 *
 * Replaces the per-minibatch body of PPO_continuous.update
 * (qiaobeibei/PPO-RL-Satellite ppo_continuous.py:213-239): actor
 * clipped-surrogate + entropy loss and critic MSE loss, their backward
 * passes, clip_grad_norm_(0.5) per net and Adam(eps) per net.  Actor and
 * critic (same hidden width H, tanh) are stepped together on the same
 * minibatch rows.  Per minibatch: satrl_ppo_rowpass (everything that is
 * row-parallel, incl. the two H x H products on f32 MFMA), satrl_ppo_dw2
 * (the dW2 weight gradient, split-K over rows), satrl_ppo_reduce and
 * satrl_ppo_adam.
 *
 * Flat parameter / gradient / Adam-moment layout (f32, see satrl_ppo_layout):
 *   W2   [2][H][H]     fc2.weight (actor, critic)
 *   W1   [2][H][20]    [fc1.weight(18) | fc1.bias | 0]  (actor, critic)
 *   b2   [2][H]        fc2.bias
 *   W3a  [3][H]        actor mean_layer.weight
 *   b3a  [4]           actor mean_layer.bias (3 used)
 *   ls   [4]           actor log_std (3 used)
 *   W3c  [H]           critic fc3.weight
 *   b3c  [4]           critic fc3.bias (1 used)
 * Gradients are produced as split-K partial slabs (dW2 from satrl_ppo_dw2
 * split S ways, [dW1|db1] and the "tail" b2..b3c (6H+12 floats) from
 * satrl_ppo_rowpass) and summed by satrl_ppo_reduce in a fixed order, so a
 * step is bitwise deterministic.  Packed transition rows (src) are [B][32] f32:
 * s(18) a(3) logp(3) adv(1) v_target(1) pad(6).
 */
#ifndef SATRL_PPO_H
#define SATRL_PPO_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { SATRL_PPO_OFF_W2 = 0, SATRL_PPO_OFF_W1, SATRL_PPO_OFF_B2, SATRL_PPO_OFF_W3A, SATRL_PPO_OFF_B3A,
       SATRL_PPO_OFF_LS, SATRL_PPO_OFF_W3C, SATRL_PPO_OFF_B3C, SATRL_PPO_TOTAL, SATRL_PPO_NOFF };

/* host helper: element offsets of the flat layout for hidden width H (64, 128 or 256) */
int satrl_ppo_layout(int H, int64_t* offsets /* [SATRL_PPO_NOFF] */);
/* number of partial slabs (row blocks: 32 rows, or 16 at H = 256 for mb <= 1024) the rowpass of a
 * minibatch of mb rows -- or of any shorter one -- writes, and of norm blocks */
int satrl_ppo_sizes(int H, int mb, int64_t* n_head_wg, int64_t* n_norm_blocks);

/* `net` (rowpass, reduce, adam): -1 = actor and critic in one launch, 0 =
 * actor only, 1 = critic only.  The two nets share nothing in a minibatch
 * step but the rows, and a one-net call touches only that net's elements
 * of every buffer, so the actor and critic chains may run concurrently on
 * two streams (each with its own nsq buffer).                              */

/* dW2 = dZ2^T H1 per net (the fc2 weight gradient) split-K S ways into the
 * slabs p2 [2][S][H][H] (f32 MFMA, fixed summation order) from the f32 rows
 * satrl_ppo_rowpass writes, at every width.  S must be
 * satrl_ppo_dw2_splits(H, mb) (about one workgroup per CU, no empty split).
 * The product paths: H = 64 / 128 fuse the product into the rowpass
 * (satrl_ppo_rowpass_dw2), H = 256 runs it from k-packed planes
 * (satrl_ppo_rowpass_kx + satrl_ppo_dw2_kx).                              */
int satrl_ppo_dw2_splits(int H, int mb);
/* Capacities (every call that writes or reads the dW2 slabs or the k-packed
 * planes takes the caller's buffer size and refuses with -1, before any
 * launch, when the call would run past it): p2_floats = elements of p2,
 * at least (net == 0 ? 1 : 2) * S * H * H; kx_elems = elements of EACH of
 * H1x / dZ2x, at least satrl_ppo_kx_elems(H, mb) (half of it for net 0).  */
int satrl_ppo_dw2(int H, int mb, int net, int S, const float* H1, const float* dZ2, float* p2, int64_t p2_floats,
                  void* stream);

/* mode 1: sum the partial slabs into G (p2: dW2 split-K [2][S][H][H], p1:
 * satrl_ppo_rowpass [dW1|db1] slabs, pt: satrl_ppo_rowpass tail slabs); mode 2: per-block
 * sums of squares of G per net into nsq [n_norm_blocks][2] (f64) and
 * advance steps [net] (f64); mode 3: both.  (mode 1 | all-reduce(G) | mode 2
 * under data parallelism.)  Every sum has a fixed order.  Mode bit 4 (with
 * 1 or 3): the W2 region only, after satrl_ppo_dw2_kx_w1 summed the W1 and
 * tail regions (p1 / pt may then be NULL).                                 */
int satrl_ppo_reduce(int H, int mb, int net, int S, int mode, const float* p2, int64_t p2_floats, const float* p1,
                     const float* pt, float* G, double* nsq, double* steps, void* stream);

/* Data parallelism, after the all-reduce (SUM) of G over `world` ranks:
 * G /= world (IEEE division, = torch's div_ of the gradient average), then
 * satrl_ppo_reduce mode 2 on it.  One launch, so mode 1 | ncclAllReduce |
 * this | satrl_ppo_adam is a single-stream chain a hipGraph captures whole.
 * Replaces the per-minibatch gradient of PPO_continuous.update
 * (ppo_continuous.py:227-239) for a minibatch spread over the ranks.       */
int satrl_ppo_reduce_dp(int H, int mb, int net, int world, float* G, double* nsq, double* steps, void* stream);

/* clip_grad_norm_(max_norm) per net (use_clip) + torch Adam (lerp form) per
 * net: lr [2] f32 device; bct f64 [bct_len][2] = {1 - beta1**k, sqrt(1 -
 * beta2**k)} for step k computed on the host with python-float math (as
 * torch.optim.Adam does), 1.0 past the table.                             */
int satrl_ppo_adam(int H, int mb, int net, const double* nsq, const double* steps, const double* bct, int bct_len,
                   const float* lr, float beta1, float beta2, float eps, float max_norm, int use_clip, const float* G,
                   float* P, float* M, float* V, void* W2X /* nullable: also refresh the fc2 operand image */,
                   void* stream);

/* The fc2 operand image W2X the rowpass reads for its two H x H products
 * (and satrl_ppo_adam keeps current), satrl_ppo_w2x_floats(H) floats: the
 * f32 fc2.weight^T per net, [2][H][H], at every width (phase D's B operand;
 * at H = 256 the rowpass splits it into bf16 planes in registers -- a
 * pre-split planes image measured slower).
 * satrl_ppo_w2x_sync builds it from P (net -1: both) -- after a load or any
 * write to fc2.weight outside satrl_ppo_adam.                               */
int64_t satrl_ppo_w2x_floats(int H);
int satrl_ppo_w2x_sync(int H, int net, const float* P, void* W2X, void* stream);

/* The row-parallel part of one minibatch step in ONE launch (a workgroup
 * per net and 32-row block): gather + fc1 + tanh, fc2 (f32 MFMA; split-bf16
 * at H = 256), output layer, the net's loss and gradients, backprop through
 * fc2 (the fc2 operand image W2X, above) and tanh(fc1).  Rows are
 * src[idx[r]] (idx nullable: rows 0..mb-1 of src, contiguous).  Writes H1
 * and dZ2 [2][mb][H] (inputs of the dW2 GEMM), the tail partial slabs
 * [n_head_wg][6H+12] and the [dW1 | db1] partial slabs [n_head_wg][2][H][20]
 * (n_head_wg from satrl_ppo_sizes).                                      */
int satrl_ppo_rowpass(int H, int mb, int net, const float* src, const int64_t* idx, const float* P, const void* W2X,
                      float epsilon, float ent_coef, float max_action, float* H1, float* dZ2, float* ptail,
                      float* pw1, void* stream);

/* The same launch for the actor's probability ratios: ratio f32 [mb]
 * (row order of the minibatch) receives exp(logp(a|s) - logp_old) of every
 * row as the loss head computes it (ppo_continuous.py:220); the other
 * outputs are satrl_ppo_rowpass's.  The parity hook of the identity "the
 * first epoch's first minibatch recomputes the rollout's log-probs bit for
 * bit", i.e. every ratio == 1.0f exactly.  net must include the actor.    */
int satrl_ppo_rowpass_ratio(int H, int mb, int net, const float* src, const int64_t* idx, const float* P,
                            const void* W2X, float epsilon, float ent_coef, float max_action, float* H1, float* dZ2,
                            float* ptail, float* pw1, float* ratio, void* stream);

/* H = 64 / 128 (BASELINE configs[1]): the rowpass with the dW2 product fused
 * in.  Each workgroup multiplies its own 32 rows' dZ2^T H1 out of LDS and
 * writes that partial as split-K slab (its row block) of p2 [2][S][H][H],
 * S = satrl_ppo_row_blocks(H, mb); H1 / dZ2 are not written.  The slabs are
 * bitwise satrl_ppo_dw2's at that S (one 32-row chunk per split, the same
 * MFMA sequence), so satrl_ppo_reduce(..., S, ...) gives the same G; the
 * minibatch step is three launches (rowpass_dw2, reduce, adam).            */
int satrl_ppo_row_blocks(int H, int mb);
int satrl_ppo_rowpass_dw2(int H, int mb, int net, const float* src, const int64_t* idx, const float* P,
                          const void* W2X, float epsilon, float ent_coef, float max_action, float* p2,
                          int64_t p2_floats /* >= (net == 0 ? 1 : 2) * S * H * H */, float* ptail, float* pw1,
                          void* stream);

/* H = 256, every minibatch (32-row workgroups above 1024 rows, 16-row ones
 * up to it): the rowpass with H1 and dZ2 written as k-packed bf16 planes (each element split hi + mid +
 * lo exactly; element (r, n) of a net's plane at ((r/8)*H + n)*8 + r%8,
 * rows padded with zeros to whole 32-row chunks): u16 H1x / dZ2x
 * [2][3][ceil(mb/32)*32][H], satrl_ppo_kx_elems(H, mb) elements each.
 * satrl_ppo_dw2_kx multiplies them into the dW2 split-K slabs p2
 * [2][S][H][H] on the split-bf16 MFMA (the fc2 products' arithmetic: error
 * below an f32 MFMA chain's), S = satrl_ppo_dw2_kx_splits(H, mb, net); the
 * minibatch step is then rowpass_kx, dw2_kx, reduce(S), adam.              */
int64_t satrl_ppo_kx_elems(int H, int mb);
int satrl_ppo_rowpass_kx(int H, int mb, int net, const float* src, const int64_t* idx, const float* P, const void* W2X,
                         float epsilon, float ent_coef, float max_action, void* H1x, void* dZ2x, int64_t kx_elems,
                         float* ptail, float* pw1, void* stream);
int satrl_ppo_dw2_kx_splits(int H, int mb, int net);
int satrl_ppo_dw2_kx(int H, int mb, int net, int S, const void* H1x, const void* dZ2x, int64_t kx_elems, float* p2,
                     int64_t p2_floats, void* stream);
/* satrl_ppo_dw2_kx and satrl_ppo_reduce's W1 / tail regions in one launch
 * (their slabs p1 / pt are the rowpass's, ready before dW2 runs): G's W1 and
 * tail parts, and with mode 3 their squared-norm pairs in nsq; then
 * satrl_ppo_reduce(..., mode | 4, ...) sums the W2 region.  Bitwise the
 * dw2_kx + reduce(mode) pair.  mode 1 or 3.                                */
int satrl_ppo_dw2_kx_w1(int H, int mb, int net, int S, const void* H1x, const void* dZ2x, int64_t kx_elems, float* p2,
                        int64_t p2_floats, int mode, const float* p1, const float* pt, float* G, double* nsq,
                        void* stream);
/* Up to 1024 rows (configs[3]'s per-rank minibatch, the 16-row range),
 * both nets, when its grid is resident at once, satrl_ppo_rowpass_kx runs
 * the column-split kernel: each (16-row block, net) on four workgroups of
 * four waves, one per 64 hidden columns, which exchange the output-layer
 * partials and the dZ2
 * planes inside the launch (bitwise the 16-wave kernel's outputs).  Its
 * exchange state is the library's own, per device: launches of it must not
 * run concurrently on two streams of one device.  A wait that times out
 * (0.5 s; a grid not co-resident) leaves the kernel with its outputs invalid
 * and sets an error word: satrl_ppo_rowpass_error waits for the stream
 * (at most timeout_s seconds of host time: -2 when it has not drained by
 * then, e.g. behind a collective of a dead peer), reports the word in *err
 * (1; 0 = none), and on an error re-arms the exchange state (the update
 * that saw it must be discarded).                                          */
int satrl_ppo_rowpass_error(int* err, double timeout_s, void* stream);
/* Fault injection for tests: sets (row block, net) group `group`'s exchange
 * counter to `value` (synchronising the stream).  A value that breaks the
 * counter's invariant (a multiple of 8 at every launch's start, e.g. 5)
 * makes that group's next launch wait out its timeout, set the error word
 * and leave the kernel: the path satrl_ppo_rowpass_error reports.        */
int satrl_ppo_rowpass_fault_inject(int group, unsigned value, void* stream);

/* Rollout forward passes on the rowpass's own MLP code, so every row's result
 * is independent of N and of the sharding, and the rollout's log-probs equal
 * the update's first recomputation bit for bit.
 * satrl_policy_act <- CPPO_main.py:122-123 (both agents' choose_action,
 * ppo_continuous.py:176-189): for the actor (net 0) of each flat parameter
 * set P0 (pursuer, agent 0) and P1 (evader, agent 1; nullable = one agent),
 * mean = max_action*tanh(mean_layer), a = clamp(mean + exp(log_std)*z,
 * +-max_action), per-dim Normal log-prob; z from Philox4x32-10 keyed by
 * (seed, agent, env_offset + row, step + *step_base) exactly as
 * satrl_gaussian_sample.  obs f32 [N][18], act/logp f32 [N][3].           */
int satrl_policy_act(int H, int64_t N, const float* obs, const float* P0, const float* P1, float max_action,
                     uint64_t seed, int64_t env_offset, uint64_t step, const uint64_t* step_base, float* act0,
                     float* logp0, float* act1, float* logp1, void* stream);
/* critic value v f32 [N] of the flat parameters P (net 1) <- self.critic(s),
 * ppo_continuous.py:200-201                                               */
int satrl_policy_value(int H, int64_t N, const float* obs, const float* P, float* v_out, void* stream);

/* Minibatch staging for a graph-replayed group of minibatches
 * (BatchSampler(SubsetRandomSampler) order, ppo_continuous.py:217): rows
 * [0, rows) of stage f32 [rows][32] = src[perm[group[0] * rows + r]] (packed
 * transition rows, 32 f32 each), with group a device i64 counter, so the
 * replayed graph walks the epoch's permutation without a host copy.
 * satrl_ppo_group_advance: group[0] += 1 (the last node of such a graph).  */
int satrl_ppo_stage(int64_t rows, const float* src, const int64_t* perm, const int64_t* group, float* stage,
                    void* stream);
int satrl_ppo_group_advance(int64_t* group, void* stream);

/* y[i] = tanh(x[i]) f32 [n], with the activation every MLP kernel above uses
 * for torch.tanh in Actor_Gaussian / Critic.forward (ppo_continuous.py:61-134):
 * the hook of its exhaustive accuracy test.                               */
int satrl_ppo_tanh(int64_t n, const float* x, float* y, void* stream);

/* Live launch spans (measurement only; bench.py): while a probe buffer is
 * set, every launch of the rowpass, dW2 (k-packed), reduce, Adam, policy /
 * value and env-step (satenv.h) kernels -- eager or captured into a graph --
 * runs the kernel's SPAN instantiation, which differs from the product one
 * only in that lane 0 of every wave stores the wave's (start, exit)
 * s_memrealtime pair (100 MHz) into a region of the buffer of its own: 2
 * u64 per wave, regions taken in launch order.  A graph captured meanwhile
 * keeps its regions: each replay rewrites them.  satrl_span_probe(buf,
 * bytes, stream) zeroes buf on `stream` and starts the log; (NULL, 0) stops
 * probing (launches run the product instantiations again).  Launch i of the
 * log: its kernel kind (0 rowpass, 1 dW2, 2 reduce, 3 Adam, 4 policy_act, 5
 * policy_value, 6 env step), the u64 offset of its records and its wave
 * count; its span = max(exit) - min(start) over its waves.                */
int satrl_span_probe(void* buf, int64_t bytes, void* stream);
int64_t satrl_span_probe_launches(void);
int satrl_span_probe_launch(int64_t i, int* kind, int64_t* word_offset, int64_t* waves);

const char* satrl_ppo_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
