/*
 * satrl_peer.h -- C ABI of the peer (IPC / xGMI) gradient all-reduce of the
 * data-parallel minibatch step (gfx950).
 *
 * Replaces, for W ranks of one node, the per-minibatch gradient averaging of
 * a data-parallel PPO_continuous.update (ppo_continuous.py:227-239 run on a
 * minibatch spread over the ranks): a deterministic two-shot
 * reduce-scatter + all-gather of the flat gradient G over buffers every rank
 * maps with hipIpcOpenMemHandle, fused with satrl_ppo_reduce_dp.  It is the
 * alternative to ncclAllReduce + satrl_ppo_reduce_dp, capturable in the
 * update's hipGraphs, and bitwise identical on every rank.
 *
 * Protocol: each value travels as one 8-byte {tag, f32} granule written by
 * a single system-scope store and polled by its reader; the tag is the call
 * count (per-block counters kept in each rank's own buffer), so no flag,
 * fence, memset or barrier is needed between calls.  A slice is summed by
 * its owner in rank order 0..W-1, divided by W, and broadcast.
 */
#ifndef SATRL_PEER_H
#define SATRL_PEER_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { SATRL_PEER_HANDLE_BYTES = 64, SATRL_PEER_MAX_WORLD = 8 };

/* bytes of one rank's exchange buffer for n floats over `world` ranks */
int satrl_peer_buffer_bytes(int64_t n, int world, int64_t* bytes);
/* allocate this rank's buffer (uncached device memory, zeroed) and its IPC
 * handle (SATRL_PEER_HANDLE_BYTES bytes, to be sent to every peer)          */
int satrl_peer_alloc(int64_t bytes, void** buf, void* ipc_handle);
/* map a peer's buffer from its handle / unmap it; free this rank's own     */
int satrl_peer_open(const void* ipc_handle, void** buf);
int satrl_peer_close(void* buf);
int satrl_peer_free(void* buf);
/* this rank's sticky error word, read after the calls queued on `stream`
 * (the call synchronises that stream): nonzero once a call ran past its
 * deadline waiting for a peer's granule (its result and every later one are
 * invalid until satrl_peer_reset)                                          */
int satrl_peer_error(const void* buf, uint64_t* err, void* stream);
/* re-arm this rank's buffer (`bytes` from satrl_peer_buffer_bytes): zero its
 * call counters, slots and error word.  Every rank resets its own buffer,
 * and no rank calls satrl_ppo_allreduce_peer again before all have (a
 * barrier), so the ranks' call counters agree again                        */
int satrl_peer_reset(void* buf, int64_t bytes, void* stream);
/* the grid of satrl_ppo_allreduce_peer at width H on the current device:
 * reduce_dp's block count capped at one block per CU (every block spins
 * until its peers' values arrive, so all of them must be resident, and one
 * wave per SIMD leaves room for other streams' kernels).  Every rank must
 * pass the same count (PeerComm takes the minimum over the ranks).         */
int satrl_peer_blocks(int H, int* blocks);

/* G [layout total] f32 on every rank -> (sum over ranks in rank order) / world,
 * identical bits on every rank, then satrl_ppo_reduce_dp mode 2's per-block
 * squared norms into nsq and steps += 1 (both nets): the call replaces
 * ncclAllReduce(G) + satrl_ppo_reduce_dp(H, mb, -1, world, ...) before
 * satrl_ppo_adam.  bufs: host array of `world` device pointers, bufs[r] = rank
 * r's buffer as mapped in this process (bufs[rank] = this rank's own).
 * blocks: the grid (satrl_peer_blocks; refused when not all resident).
 * timeout_s: how long a wait for a peer's value may last before the call
 * gives up and sets the error word (the data-parallel timeout, e.g.
 * SATRL_DP_TIMEOUT_S: ranks may drift apart by host work between updates).
 * All ranks must make the same sequence of calls with the same grid.      */
int satrl_ppo_allreduce_peer(int H, int mb, int world, int rank, void* const* bufs, float* G, double* nsq,
                             double* steps, int blocks, double timeout_s, void* stream);

#ifdef __cplusplus
}
#endif
#endif
