// rub_mimo_amd/csrc/ring.cpp -- pinned-host capture ring (include/mimo_rx.h).
//
// The reference's rx worker (mimo/main.cc:842-918) recv()s fc32 into malloc'd per-channel
// buffers, appends them to /tmp/rx<ch>.dat, and reads the whole file back into one host array
// before framesync::execute. Here the recv loop writes the sc16 wire samples into chunks of one
// pinned allocation and each commit becomes a single asynchronous 2-D host-to-device copy into
// the bound device capture: 4 B per sample over PCIe (not 8), no file round trip, and the
// capture is already in the batch layout that the S&C, search + LS and streaming decode
// kernels read in place (mimo_batch.sample_format = MIMO_SAMPLE_SC16).
//
// Ordering. All uploads go through the ring's own non-blocking stream, so they complete in
// commit order and the event recorded after the latest commit stands for all of them; publish
// makes the consumer's stream wait for it on the device (no host synchronisation). A chunk's
// own event gates its reuse: acquire blocks on it, so with n_chunks >= 2 the producer fills
// chunk k + 1 while chunk k is in flight.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mimo_rx.h"
#include "kernels.hpp"

using mimo::host_fail;

struct mimo_ring {
  uint32_t n_ant = 0, chunk = 0, n_chunks = 0;
  int16_t *host = nullptr;              // pinned [n_chunks][n_ant][chunk][2]
  std::vector<hipEvent_t> done;         // per chunk: its latest upload has completed
  std::vector<char> used;               // the chunk's event has been recorded
  hipStream_t copy = nullptr;
  uint32_t next = 0;                    // chunk handed out by the next acquire
  int32_t held = -1;                    // acquired, not yet committed
  std::mutex mu;                        // bind / commit / publish
  char *cap = nullptr;                  // bound capture (sc16)
  uint64_t stride = 0, capacity = 0, pos = 0;
  hipEvent_t last = nullptr;            // the latest commit's event (nullptr: none yet)
  hipEvent_t consumed = nullptr;        // bind_after: the consumer's work on a rebound capture
};

#define RCHK(x, what)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess)                                                              \
      return host_fail(MIMO_ERR_HIP, (std::string(what) + ": " + hipGetErrorString(e_)).c_str()); \
  } while (0)

static void ring_free(mimo_ring *r) {
  if (r->copy) (void)hipStreamSynchronize(r->copy);
  for (hipEvent_t e : r->done)
    if (e) (void)hipEventDestroy(e);
  if (r->consumed) (void)hipEventDestroy(r->consumed);
  if (r->copy) (void)hipStreamDestroy(r->copy);
  if (r->host) (void)hipHostFree(r->host);
  delete r;
}

extern "C" int mimo_ring_create(uint32_t n_ant, uint32_t chunk_samples, uint32_t n_chunks,
                                mimo_ring **out) {
  if (!out) return host_fail(MIMO_ERR_ARG, "mimo_ring_create: null argument");
  *out = nullptr;
  if (n_ant == 0 || n_ant > MIMO_MAX_STREAMS || chunk_samples == 0 || n_chunks == 0)
    return host_fail(MIMO_ERR_ARG, "mimo_ring_create: need 1..8 antennas, chunks of >= 1 sample");
  const uint64_t bytes = (uint64_t)n_chunks * n_ant * chunk_samples * 4;
  if (bytes > (1ull << 36)) return host_fail(MIMO_ERR_ARG, "mimo_ring_create: ring above 64 GiB");
  mimo_ring *r = new mimo_ring;
  r->n_ant = n_ant;
  r->chunk = chunk_samples;
  r->n_chunks = n_chunks;
  r->done.assign(n_chunks, nullptr);
  r->used.assign(n_chunks, 0);
  hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&r->host), bytes, hipHostMallocDefault);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&r->copy, hipStreamNonBlocking);
  for (uint32_t k = 0; e == hipSuccess && k < n_chunks; k++)
    e = hipEventCreateWithFlags(&r->done[k], hipEventDisableTiming);
  if (e != hipSuccess) {
    ring_free(r);
    return host_fail(MIMO_ERR_HIP, (std::string("mimo_ring_create: ") + hipGetErrorString(e)).c_str());
  }
  *out = r;
  return MIMO_OK;
}

extern "C" int mimo_ring_destroy(mimo_ring *r) {
  if (!r) return host_fail(MIMO_ERR_ARG, "mimo_ring_destroy: null ring");
  ring_free(r);
  return MIMO_OK;
}

extern "C" int mimo_ring_bind(mimo_ring *r, void *d_capture, uint64_t stride, uint64_t capacity) {
  if (!r || !d_capture) return host_fail(MIMO_ERR_ARG, "mimo_ring_bind: null argument");
  if (capacity > stride && r->n_ant > 1)
    return host_fail(MIMO_ERR_ARG, "mimo_ring_bind: capacity exceeds the row stride");
  std::lock_guard<std::mutex> lk(r->mu);
  r->cap = static_cast<char *>(d_capture);
  r->stride = stride;
  r->capacity = capacity;
  r->pos = 0;
  return MIMO_OK;
}

// Write-after-read ordering for a rebound capture: the copy stream waits, on the device, for
// everything enqueued on consumer_stream so far (e.g. the batch still reading the capture)
// before the first upload of the new binding.
extern "C" int mimo_ring_bind_after(mimo_ring *r, void *d_capture, uint64_t stride,
                                    uint64_t capacity, void *consumer_stream) {
  int rc = mimo_ring_bind(r, d_capture, stride, capacity);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(r->mu);
  if (!r->consumed)
    RCHK(hipEventCreateWithFlags(&r->consumed, hipEventDisableTiming), "mimo_ring_bind_after");
  RCHK(hipEventRecord(r->consumed, (hipStream_t)consumer_stream), "mimo_ring_bind_after");
  RCHK(hipStreamWaitEvent(r->copy, r->consumed, 0), "mimo_ring_bind_after");
  return MIMO_OK;
}

extern "C" int mimo_ring_acquire(mimo_ring *r, void **rows, uint32_t *max_samples) {
  if (!r || !rows) return host_fail(MIMO_ERR_ARG, "mimo_ring_acquire: null argument");
  if (r->held >= 0) return host_fail(MIMO_ERR_ARG, "mimo_ring_acquire: previous chunk not committed");
  const uint32_t k = r->next;
  if (r->used[k]) RCHK(hipEventSynchronize(r->done[k]), "mimo_ring_acquire");
  for (uint32_t a = 0; a < r->n_ant; a++)
    rows[a] = r->host + ((uint64_t)k * r->n_ant + a) * r->chunk * 2;
  if (max_samples) *max_samples = r->chunk;
  r->held = (int32_t)k;
  return MIMO_OK;
}

extern "C" int mimo_ring_commit(mimo_ring *r, uint32_t n) {
  if (!r) return host_fail(MIMO_ERR_ARG, "mimo_ring_commit: null ring");
  if (r->held < 0) return host_fail(MIMO_ERR_ARG, "mimo_ring_commit: no chunk acquired");
  if (n > r->chunk) return host_fail(MIMO_ERR_ARG, "mimo_ring_commit: more samples than a chunk");
  const uint32_t k = (uint32_t)r->held;
  std::lock_guard<std::mutex> lk(r->mu);
  if (!r->cap) return host_fail(MIMO_ERR_ARG, "mimo_ring_commit: no capture bound");
  if (r->pos + n > r->capacity)
    return host_fail(MIMO_ERR_ARG, "mimo_ring_commit: capture full (bind the next one)");
  if (n > 0) {
    RCHK(hipMemcpy2DAsync(r->cap + r->pos * 4, r->stride * 4,
                          r->host + (uint64_t)k * r->n_ant * r->chunk * 2, (size_t)r->chunk * 4,
                          (size_t)n * 4, r->n_ant, hipMemcpyHostToDevice, r->copy),
         "mimo_ring_commit");
    RCHK(hipEventRecord(r->done[k], r->copy), "mimo_ring_commit");
    r->used[k] = 1;
    r->last = r->done[k];
    r->pos += n;
  }
  r->held = -1;
  r->next = (k + 1) % r->n_chunks;
  return MIMO_OK;
}

extern "C" int mimo_ring_publish(mimo_ring *r, void *hip_stream, uint64_t *n_written) {
  if (!r) return host_fail(MIMO_ERR_ARG, "mimo_ring_publish: null ring");
  std::lock_guard<std::mutex> lk(r->mu);
  if (r->last) RCHK(hipStreamWaitEvent((hipStream_t)hip_stream, r->last, 0), "mimo_ring_publish");
  if (n_written) *n_written = r->pos;
  return MIMO_OK;
}
