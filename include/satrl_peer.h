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
/* this rank's sticky error word (synchronous copy): nonzero after a call in
 * which a peer's granule never arrived within 0.5 s (its result is invalid) */
int satrl_peer_error(const void* buf, uint64_t* err);

/* G [layout total] f32 on every rank -> (sum over ranks in rank order) / world,
 * identical bits on every rank, then satrl_ppo_reduce_dp mode 2's per-block
 * squared norms into nsq and steps += 1 (both nets): the call replaces
 * ncclAllReduce(G) + satrl_ppo_reduce_dp(H, mb, -1, world, ...) before
 * satrl_ppo_adam.  bufs: host array of `world` device pointers, bufs[r] = rank
 * r's buffer as mapped in this process (bufs[rank] = this rank's own).  All
 * ranks must make the same sequence of calls.                              */
int satrl_ppo_allreduce_peer(int H, int mb, int world, int rank, void* const* bufs, float* G, double* nsq,
                             double* steps, void* stream);

#ifdef __cplusplus
}
#endif
#endif
