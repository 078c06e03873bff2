// rtg_comm.cpp — multi-GPU frames of the C-ABI (include/rtgpu.h "multi-GPU frames"):
// row-interleaved shards, one RCCL gather over xGMI to the root, a de-interleave kernel there.
//
// Replaces, for an image tiled over the GPUs of one node (BASELINE config 5), the
// reference's single pixel loop camera::render (src/core/camera.hpp:29-72). Rank r renders image
// rows r, r+N, ... (interleaved: sky and ground rows are dealt evenly), padded to P = ceil(H/N) rows
// so every rank sends the same P*row_bytes bytes; ncclGather lands rank r's block at r*P rows of a
// staging buffer on the root; deinterleave_kernel then writes block r row k to image row r + k*N.
// The frame is the same for any N (the render RNG is keyed by the global pixel id).
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "rtg_internal.hpp"

using namespace rtg;

namespace {

rtg_status hip_err(hipError_t e, const char* what) {
  return set_last_error(e == hipErrorOutOfMemory ? RTG_E_NOMEM : RTG_E_HIP,
                        std::string(what) + ": " + hipGetErrorString(e));
}
rtg_status nccl_err(ncclResult_t r, const char* what) {
  return set_last_error(RTG_E_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}

#define COMM_HIP(call, what)                      \
  do {                                            \
    hipError_t e_ = (call);                       \
    if (e_ != hipSuccess) return hip_err(e_, what); \
  } while (0)
#define COMM_NCCL(call, what)                          \
  do {                                                 \
    ncclResult_t r_ = (call);                          \
    if (r_ != ncclSuccess) return nccl_err(r_, what);  \
  } while (0)

// One thread per 16-byte chunk of an output row (rows of a multiple of 16 bytes: every frame
// format here, W*12 for fp32 RGB and W*3 for RGB8 with W a multiple of 16), else per byte.
// HBM-bound copy: each byte is read once and written once.
template <typename T>
__global__ __launch_bounds__(256) void deinterleave_kernel(const T* __restrict__ gathered, T* __restrict__ out,
                                                           int32_t nranks, int32_t padded, int32_t height,
                                                           int64_t row_elems) {
  const int64_t total = static_cast<int64_t>(height) * row_elems;
  for (int64_t k = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; k < total;
       k += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t row = k / row_elems, col = k - row * row_elems;
    out[k] = gathered[gathered_row(row, nranks, padded) * row_elems + col];  // image row r + j*nranks
  }
}

hipError_t launch_deinterleave(const void* gathered, void* out, int32_t nranks, int32_t height, int64_t row_bytes,
                               hipStream_t stream) {
  if (height <= 0 || row_bytes <= 0) return hipSuccess;
  const int32_t padded = shard_layout(height, nranks, 0).padded_rows;
  const bool wide = row_bytes % 16 == 0 && reinterpret_cast<uintptr_t>(gathered) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(out) % 16 == 0;
  const int64_t elems = wide ? row_bytes / 16 : row_bytes;
  const int64_t total = static_cast<int64_t>(height) * elems;
  const unsigned blocks = static_cast<unsigned>(std::min<int64_t>((total + 255) / 256, 65536));
  if (wide)
    hipLaunchKernelGGL(deinterleave_kernel<uint4>, dim3(blocks), dim3(256), 0, stream,
                       static_cast<const uint4*>(gathered), static_cast<uint4*>(out), nranks, padded, height, elems);
  else
    hipLaunchKernelGGL(deinterleave_kernel<uint8_t>, dim3(blocks), dim3(256), 0, stream,
                       static_cast<const uint8_t*>(gathered), static_cast<uint8_t*>(out), nranks, padded, height,
                       elems);
  return hipGetLastError();
}

}  // namespace

struct rtg_comm {
  int32_t nranks = 0;
  std::vector<int32_t> ranks, devices;  // per local rank
  std::vector<ncclComm_t> comms;
  std::vector<hipStream_t> streams;     // the communicator's own stream per local rank
  // scratch, grown on demand and kept: per-rank shard buffers and the root frame of rtg_render_frame, and
  // the root's gather staging buffer (rtg_gather_rows), so steady-state frames allocate nothing (VERDICT
  // r05 item 4). `stage_done` is recorded behind each gather's de-interleave: a gather on another stream
  // first waits for it, so gathers in flight on two streams take turns at the buffer instead of sharing it.
  std::vector<void*> shard;
  std::vector<size_t> shard_bytes;
  void* frame = nullptr;
  size_t frame_bytes = 0;
  int32_t frame_local = -1;  // local rank whose device holds `frame`
  void* stage = nullptr;
  size_t stage_bytes = 0;
  int32_t stage_local = -1;       // local rank whose device holds `stage`
  hipEvent_t stage_done = nullptr;  // on stage_local's device; recorded once a gather used the buffer
  bool stage_used = false;

  int32_t local_of(int32_t rank) const {
    for (size_t i = 0; i < ranks.size(); ++i)
      if (ranks[i] == rank) return static_cast<int32_t>(i);
    return -1;
  }
};

namespace {

rtg_status comm_finish(rtg_comm* c, rtg_comm** out) {
  c->shard.assign(c->ranks.size(), nullptr);
  c->shard_bytes.assign(c->ranks.size(), 0);
  c->streams.assign(c->ranks.size(), nullptr);
  for (size_t i = 0; i < c->ranks.size(); ++i) {
    hipError_t e = hipSetDevice(c->devices[i]);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->streams[i], hipStreamNonBlocking);
    if (e != hipSuccess) {
      rtg_comm_destroy(c);
      return hip_err(e, "hipStreamCreate(comm)");
    }
  }
  *out = c;
  return RTG_OK;
}

// grow a device buffer on `device` to at least `bytes`
rtg_status ensure(void** p, size_t* have, size_t bytes, int32_t device, const char* what) {
  if (*have >= bytes && *p) return RTG_OK;
  COMM_HIP(hipSetDevice(device), "hipSetDevice");
  if (*p) COMM_HIP(hipFree(*p), "hipFree(comm scratch)");
  *p = nullptr;
  *have = 0;
  COMM_HIP(dev_alloc(p, std::max<size_t>(bytes, 16)), what);
  *have = bytes;
  return RTG_OK;
}

int32_t device_count() {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

}  // namespace

extern "C" {

rtg_status rtg_comm_create_local(const int32_t* devices, int32_t ndev, rtg_comm** out) {
  if (!devices || ndev <= 0 || !out) return set_last_error(RTG_E_INVALID, "null argument or no devices");
  *out = nullptr;
  const int32_t n = device_count();
  if (n <= 0) return set_last_error(RTG_E_NODEVICE, "no HIP device available");
  for (int32_t i = 0; i < ndev; ++i)
    if (devices[i] < 0 || devices[i] >= n) return set_last_error(RTG_E_INVALID, "device index out of range");
  rtg_comm* c = new rtg_comm();
  c->nranks = ndev;
  c->devices.assign(devices, devices + ndev);
  c->comms.assign(ndev, nullptr);
  for (int32_t i = 0; i < ndev; ++i) c->ranks.push_back(i);
  const ncclResult_t r = ncclCommInitAll(c->comms.data(), ndev, c->devices.data());
  if (r != ncclSuccess) {
    c->comms.clear();
    delete c;
    return nccl_err(r, "ncclCommInitAll");
  }
  return comm_finish(c, out);
}

rtg_status rtg_comm_unique_id(uint8_t id[RTG_COMM_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) <= RTG_COMM_ID_BYTES, "ncclUniqueId larger than RTG_COMM_ID_BYTES");
  if (!id) return set_last_error(RTG_E_INVALID, "null argument");
  ncclUniqueId u;
  COMM_NCCL(ncclGetUniqueId(&u), "ncclGetUniqueId");
  std::memset(id, 0, RTG_COMM_ID_BYTES);
  std::memcpy(id, &u, sizeof(u));
  return RTG_OK;
}

rtg_status rtg_comm_create_rank(const uint8_t id[RTG_COMM_ID_BYTES], int32_t nranks, int32_t rank, int32_t device,
                                rtg_comm** out) {
  if (!id || !out || nranks <= 0 || rank < 0 || rank >= nranks)
    return set_last_error(RTG_E_INVALID, "bad communicator arguments");
  *out = nullptr;
  const int32_t n = device_count();
  if (n <= 0) return set_last_error(RTG_E_NODEVICE, "no HIP device available");
  if (device < 0 || device >= n) return set_last_error(RTG_E_INVALID, "device index out of range");
  COMM_HIP(hipSetDevice(device), "hipSetDevice");
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  rtg_comm* c = new rtg_comm();
  c->nranks = nranks;
  c->ranks.push_back(rank);
  c->devices.push_back(device);
  c->comms.assign(1, nullptr);
  const ncclResult_t r = ncclCommInitRank(&c->comms[0], nranks, u, rank);
  if (r != ncclSuccess) {
    c->comms.clear();
    delete c;
    return nccl_err(r, "ncclCommInitRank");
  }
  return comm_finish(c, out);
}

rtg_status rtg_comm_size(const rtg_comm* c, int32_t* nranks, int32_t* nlocal) {
  if (!c) return set_last_error(RTG_E_INVALID, "null communicator");
  if (nranks) {  // the rank count as RCCL itself reports it for this communicator
    int n = 0;
    if (c->comms.empty() || !c->comms[0]) return set_last_error(RTG_E_INVALID, "communicator not initialised");
    COMM_NCCL(ncclCommCount(c->comms[0], &n), "ncclCommCount");
    *nranks = n;
  }
  if (nlocal) *nlocal = static_cast<int32_t>(c->ranks.size());
  return RTG_OK;
}

void rtg_comm_destroy(rtg_comm* c) {
  if (!c) return;
  // teardown: errors cannot be reported from a void destructor, they are deliberately dropped
  for (size_t i = 0; i < c->ranks.size(); ++i) {
    (void)hipSetDevice(c->devices[i]);
    if (i < c->streams.size() && c->streams[i]) (void)hipStreamSynchronize(c->streams[i]);
    if (i < c->shard.size() && c->shard[i]) (void)hipFree(c->shard[i]);
  }
  if (c->frame) {
    (void)hipSetDevice(c->devices[c->frame_local]);
    (void)hipFree(c->frame);
  }
  if (c->stage_local >= 0) {
    (void)hipSetDevice(c->devices[c->stage_local]);
    if (c->stage) (void)hipFree(c->stage);  // hipFree waits for the device: no gather still reads it
    if (c->stage_done) (void)hipEventDestroy(c->stage_done);
  }
  for (ncclComm_t m : c->comms)
    if (m) (void)ncclCommDestroy(m);
  for (size_t i = 0; i < c->streams.size(); ++i)
    if (c->streams[i]) {
      (void)hipSetDevice(c->devices[i]);
      (void)hipStreamDestroy(c->streams[i]);
    }
  delete c;
}

rtg_status rtg_deinterleave_rows(int32_t device, const void* gathered, void* out, int32_t nranks, int32_t height,
                                 int64_t row_bytes, void* stream) {
  if (!gathered || !out || nranks <= 0 || height < 0 || row_bytes < 0)
    return set_last_error(RTG_E_INVALID, "bad de-interleave arguments");
  COMM_HIP(hipSetDevice(device), "hipSetDevice");
  COMM_HIP(launch_deinterleave(gathered, out, nranks, height, row_bytes, static_cast<hipStream_t>(stream)),
           "de-interleave kernel launch");
  return RTG_OK;
}

rtg_status rtg_shard_layout(int32_t height, int32_t nranks, int32_t rank, int32_t* row_begin, int32_t* row_stride,
                            int32_t* row_count, int32_t* padded_rows) {
  if (height <= 0 || nranks <= 0 || rank < 0 || rank >= nranks)
    return set_last_error(RTG_E_INVALID, "bad shard layout arguments");
  const ShardLayout L = shard_layout(height, nranks, rank);
  if (row_begin) *row_begin = L.row_begin;
  if (row_stride) *row_stride = L.row_stride;
  if (row_count) *row_count = L.row_count;
  if (padded_rows) *padded_rows = L.padded_rows;
  return RTG_OK;
}

rtg_status rtg_deinterleave_rows_host(const void* gathered, void* out, int32_t nranks, int32_t height,
                                      int64_t row_bytes) {
  if (!gathered || !out || nranks <= 0 || height < 0 || row_bytes < 0)
    return set_last_error(RTG_E_INVALID, "bad de-interleave arguments");
  if (height == 0) return RTG_OK;
  const int32_t padded = shard_layout(height, nranks, 0).padded_rows;
  const auto* g = static_cast<const uint8_t*>(gathered);
  auto* o = static_cast<uint8_t*>(out);
  for (int64_t row = 0; row < height; ++row)
    std::memcpy(o + row * row_bytes, g + gathered_row(row, nranks, padded) * row_bytes, static_cast<size_t>(row_bytes));
  return RTG_OK;
}

rtg_status rtg_gather_rows(rtg_comm* c, const void* const* shards, int32_t height, int64_t row_bytes, int32_t root,
                           void* out, void* const* streams) {
  if (!c || !shards || height <= 0 || row_bytes <= 0 || root < 0 || root >= c->nranks)
    return set_last_error(RTG_E_INVALID, "bad gather arguments");
  const int32_t N = c->nranks, P = shard_layout(height, N, 0).padded_rows;
  const int32_t nlocal = static_cast<int32_t>(c->ranks.size());
  const int32_t rl = c->local_of(root);
  if (rl >= 0 && !out) return set_last_error(RTG_E_INVALID, "null output on the root");
  const size_t block = static_cast<size_t>(P) * static_cast<size_t>(row_bytes);
  auto stream_of = [&](int32_t i) {
    return (streams && streams[i]) ? static_cast<hipStream_t>(streams[i]) : c->streams[i];
  };
  // the root's staging buffer, grown on demand and kept (rtg_comm::stage); the root's stream waits for the
  // previous gather's de-interleave (whatever stream that ran on) before RCCL writes into it
  void* stage = nullptr;
  if (rl >= 0) {
    COMM_HIP(hipSetDevice(c->devices[rl]), "hipSetDevice");
    const size_t need = std::max<size_t>(block * N, 16);
    if (c->stage_local != rl || c->stage_bytes < need || !c->stage) {
      if (c->stage_local >= 0) {  // regrow (or a new root): free the old buffer once nothing reads it
        COMM_HIP(hipSetDevice(c->devices[c->stage_local]), "hipSetDevice");
        if (c->stage_used) COMM_HIP(hipEventSynchronize(c->stage_done), "hipEventSynchronize(gather stage)");
        if (c->stage) COMM_HIP(hipFree(c->stage), "hipFree(gather stage)");
        if (c->stage_done) COMM_HIP(hipEventDestroy(c->stage_done), "hipEventDestroy");
        c->stage = nullptr;
        c->stage_done = nullptr;
        c->stage_bytes = 0;
        c->stage_used = false;
        c->stage_local = -1;
        COMM_HIP(hipSetDevice(c->devices[rl]), "hipSetDevice");
      }
      COMM_HIP(hipEventCreateWithFlags(&c->stage_done, hipEventDisableTiming), "hipEventCreate");
      c->stage_local = rl;
      COMM_HIP(dev_alloc(&c->stage, need), "hipMalloc(gather stage)");
      c->stage_bytes = need;
    } else if (c->stage_used) {
      COMM_HIP(hipStreamWaitEvent(stream_of(rl), c->stage_done, 0), "hipStreamWaitEvent(gather stage)");
    }
    stage = c->stage;
  }
  if (const ncclResult_t r = ncclGroupStart(); r != ncclSuccess) {
    return nccl_err(r, "ncclGroupStart");
  }
  for (int32_t i = 0; i < nlocal; ++i) {
    const hipError_t e = hipSetDevice(c->devices[i]);
    if (e != hipSuccess) {
      (void)ncclGroupEnd();
        return hip_err(e, "hipSetDevice");
    }
    const ncclResult_t r = ncclGather(shards[i], i == rl ? stage : nullptr, block, ncclUint8, root, c->comms[i],
                                      stream_of(i));
    if (r != ncclSuccess) {
      (void)ncclGroupEnd();
        return nccl_err(r, "ncclGather");
    }
  }
  if (const ncclResult_t r = ncclGroupEnd(); r != ncclSuccess) {
    return nccl_err(r, "ncclGroupEnd");
  }
  if (rl >= 0) {
    COMM_HIP(hipSetDevice(c->devices[rl]), "hipSetDevice");
    const hipError_t e = launch_deinterleave(stage, out, N, height, row_bytes, stream_of(rl));
    if (e != hipSuccess) return hip_err(e, "de-interleave kernel launch");
    COMM_HIP(hipEventRecord(c->stage_done, stream_of(rl)), "hipEventRecord(gather stage)");
    c->stage_used = true;
  }
  return RTG_OK;
}

rtg_status rtg_render_frame(rtg_comm* c, rtg_scene* const* scenes, const rtg_camera_desc* cam, uint64_t seed,
                            int32_t root, float* out_rgb, rtg_render_stats* stats) {
  if (!c || !scenes || !cam) return set_last_error(RTG_E_INVALID, "null argument");
  if (root < 0 || root >= c->nranks) return set_last_error(RTG_E_INVALID, "root outside the communicator");
  rtg_camera_params cp;
  rtg_status st = rtg_camera_resolve(cam, &cp);
  if (st != RTG_OK) return st;
  const int32_t N = c->nranks, H = cp.image_height, W = cp.image_width, P = shard_layout(H, N, 0).padded_rows;
  const int32_t nlocal = static_cast<int32_t>(c->ranks.size());
  const int64_t row_bytes = static_cast<int64_t>(W) * 3 * sizeof(float);
  for (int32_t i = 0; i < nlocal; ++i) {
    rtg_scene_info info;
    if ((st = rtg_scene_get_info(scenes[i], &info)) != RTG_OK) return st;
    if (info.device != c->devices[i])
      return set_last_error(RTG_E_INVALID, "scenes[i] is not on the communicator's i-th device");
  }
  // 1. every local rank renders its interleaved rows into its shard buffer (asynchronously)
  std::vector<const void*> shard_ptrs(nlocal);
  std::vector<void*> streams(nlocal);
  std::vector<bool> launched(nlocal, false);
  auto drain = [&]() {  // on an error: collect the renders already launched, keep the first error text
    const std::string msg = rtg_last_error();
    for (int32_t i = 0; i < nlocal; ++i)
      if (launched[i]) (void)rtg_render_wait(scenes[i], nullptr);
    return msg;
  };
  for (int32_t i = 0; i < nlocal; ++i) {
    if ((st = ensure(&c->shard[i], &c->shard_bytes[i], static_cast<size_t>(P) * row_bytes, c->devices[i],
                     "hipMalloc(shard)")) != RTG_OK) {
      const std::string msg = drain();
      return set_last_error(st, msg);
    }
    shard_ptrs[i] = c->shard[i];
    streams[i] = c->streams[i];
    const ShardLayout L = shard_layout(H, N, c->ranks[i]);
    if (L.row_count == 0) continue;  // a rank past the last row only sends padding
    rtg_render_desc job{};
    job.seed = seed;
    job.row_begin = L.row_begin;
    job.row_stride = L.row_stride;
    job.row_count = L.row_count;
    job.flags = RTG_RENDER_OUT_DEVICE | RTG_RENDER_ASYNC;
    job.stream = c->streams[i];
    if ((st = rtg_render(scenes[i], cam, &job, static_cast<float*>(c->shard[i]), nullptr)) != RTG_OK) {
      const std::string msg = drain();
      return set_last_error(st, msg);
    }
    launched[i] = true;
  }
  // 2. one RCCL gather (all local ranks in one group) + the de-interleave on the root
  const int32_t rl = c->local_of(root);
  if (rl >= 0) {
    if (c->frame && c->frame_local != rl) {
      (void)hipSetDevice(c->devices[c->frame_local]);
      (void)hipFree(c->frame);
      c->frame = nullptr;
      c->frame_bytes = 0;
    }
    c->frame_local = rl;
    if ((st = ensure(&c->frame, &c->frame_bytes, static_cast<size_t>(H) * row_bytes, c->devices[rl],
                     "hipMalloc(frame)")) != RTG_OK) {
      const std::string msg = drain();
      return set_last_error(st, msg);
    }
  }
  if ((st = rtg_gather_rows(c, shard_ptrs.data(), H, row_bytes, root, c->frame, streams.data())) != RTG_OK) {
    const std::string msg = drain();
    return set_last_error(st, msg);
  }
  // 3. wait for every rank (stats), then the frame to the host on the root's process
  rtg_render_stats total{};
  rtg_status first = RTG_OK;
  std::string first_msg;
  for (int32_t i = 0; i < nlocal; ++i) {
    if (!launched[i]) continue;
    rtg_render_stats s{};
    const rtg_status w = rtg_render_wait(scenes[i], &s);
    if (w != RTG_OK && first == RTG_OK) {
      first = w;
      first_msg = rtg_last_error();
    }
    total.segments += s.segments;
    total.samples += s.samples;
    total.box_tests += s.box_tests;
    total.prim_tests += s.prim_tests;
    total.hits += s.hits;
    total.kernel_ms = std::max(total.kernel_ms, s.kernel_ms);
  }
  if (first != RTG_OK) return set_last_error(first, first_msg);
  for (int32_t i = 0; i < nlocal; ++i) {
    COMM_HIP(hipSetDevice(c->devices[i]), "hipSetDevice");
    COMM_HIP(hipStreamSynchronize(c->streams[i]), "gather");
  }
  if (rl >= 0 && out_rgb) {
    COMM_HIP(hipSetDevice(c->devices[rl]), "hipSetDevice");
    COMM_HIP(hipMemcpy(out_rgb, c->frame, static_cast<size_t>(H) * row_bytes, hipMemcpyDeviceToHost),
             "hipMemcpy(frame)");
  }
  if (stats) *stats = total;
  return RTG_OK;
}

}  // extern "C"
