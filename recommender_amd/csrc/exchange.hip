// exchange.hip — the row-sharded slab's capacity-bounded exchange (BASELINE north
// star "tables shard row-wise across the 8 GPUs of one node with RCCL all-to-all over xGMI").
//
// Every rank sends every owner a fixed `capacity` C of row slots per step, so both all-to-alls
// of a step (row ids out, rows back; gradient rows out) move [world, C] blocks with EQUAL split
// sizes: no host sync on the counts. Two per-step sizes remain host-read — the spill round's C2
// and the rows-ahead late round's C_late, each read a step after it is known (no stall), but a
// captured graph would freeze them, so the sharded step is NOT capturable (TrainStep.capture
// raises for it).
// A rank's unique rows (owner-major sorted keys, rs_unique_inverse) are dealt to the slots in
// key order: unique u of owner o goes to slot o·C + (u − first unique of o). Slots left over are
// padding (id −1: the owner gathers a zero row and its apply leaves the slot out). Rows past C
// (a batch with more unique rows for one owner than the capacity) take a spill round: every rank
// learns the all-reduced largest excess C2 (rs_exchange_excess), and the excess rows go in a
// second pair of equal-split all-to-alls of [world, C2] blocks (rs_exchange_pack_spill) — slots
// world·C + o·C2 + j, after the capacity block (recommender_amd/sharded.py).
#include "common.hpp"

namespace rs {

// ostart[o] = first unique of owner o: an exclusive scan of owner_counts, made per block in LDS
constexpr int kMaxWorld = 1024;

__device__ __forceinline__ void owner_starts(const int32_t* counts, int world, int32_t* ostart) {
  if (threadIdx.x == 0) {
    int32_t run = 0;
    for (int o = 0; o < world; ++o) {
      ostart[o] = run;
      run += counts[o];
    }
  }
  __syncthreads();
}

// unique u → padded slot (or −1 past capacity), and the send buffer's row ids
__global__ __launch_bounds__(256) void exchange_slots_kernel(
    const uint32_t* __restrict__ uniq, const int32_t* __restrict__ n_unique,
    const int32_t* __restrict__ counts, int world, int64_t stride, int64_t cap, int64_t n_max,
    int32_t* __restrict__ send_ids, int32_t* __restrict__ slot_of, int32_t* __restrict__ overflow) {
  __shared__ int32_t ostart[kMaxWorld];
  owner_starts(counts, world, ostart);
  const int64_t U = *n_unique;
  bool over = false;
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n_max;
       u += (int64_t)gridDim.x * blockDim.x) {
    if (u >= U) break;
    const int64_t key = uniq[u];
    const int o = (int)(key / stride);
    const int64_t j = u - ostart[o];
    if (j < cap) {
      const int64_t slot = (int64_t)o * cap + j;
      send_ids[slot] = (int32_t)(key - (int64_t)o * stride);
      slot_of[u] = (int32_t)slot;
    } else {
      slot_of[u] = -1;
      over = true;
    }
  }
  if (__any(over) && (threadIdx.x & 63) == 0) atomicOr(overflow, 1);
}

// position p → the padded slot of its unique row (−1: OOB id or a row past capacity)
__global__ __launch_bounds__(256) void exchange_inverse_kernel(const int32_t* __restrict__ inverse,
                                                               const int32_t* __restrict__ slot_of,
                                                               int64_t n,
                                                               int32_t* __restrict__ inv_slot) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t u = inverse[p];
    inv_slot[p] = u >= 0 ? slot_of[u] : -1;
  }
}

// the rows past the capacity: unique u of owner o with j = u - ostart[o] >= cap goes to spill
// slot world·cap + o·cap2 + (j - cap) (cap2 >= every rank's largest excess: the all-reduced
// maximum), its local row to spill_ids[o·cap2 + j - cap]
__global__ __launch_bounds__(256) void exchange_spill_slots_kernel(
    const uint32_t* __restrict__ uniq, const int32_t* __restrict__ n_unique,
    const int32_t* __restrict__ counts, int world, int64_t stride, int64_t cap, int64_t cap2,
    int64_t n_max, int32_t* __restrict__ spill_ids, int32_t* __restrict__ slot_of,
    int32_t* __restrict__ overflow) {
  __shared__ int32_t ostart[kMaxWorld];
  owner_starts(counts, world, ostart);
  const int64_t U = *n_unique;
  bool over = false;
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n_max;
       u += (int64_t)gridDim.x * blockDim.x) {
    if (u >= U) break;
    const int64_t key = uniq[u];
    const int o = (int)(key / stride);
    const int64_t j = u - ostart[o] - cap;
    if (j < 0) continue;
    if (j < cap2) {
      spill_ids[(int64_t)o * cap2 + j] = (int32_t)(key - (int64_t)o * stride);
      slot_of[u] = (int32_t)((int64_t)world * cap + (int64_t)o * cap2 + j);
    } else {
      over = true;  // cap2 smaller than the excess: the caller passed a wrong cap2
    }
  }
  if (__any(over) && (threadIdx.x & 63) == 0 && overflow) atomicOr(overflow, 1);
}

// the largest excess over the capacity among this rank's owners: max(0, counts[o] - cap)
__global__ void exchange_excess_kernel(const int32_t* __restrict__ counts, int world, int64_t cap,
                                       int64_t* __restrict__ excess) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int64_t m = 0;
  for (int o = 0; o < world; ++o) {
    const int64_t e = (int64_t)counts[o] - cap;
    m = e > m ? e : m;
  }
  *excess = m;
}

// the owner's side: out[i] = shard[ids[i]] for ids in range, a zero row for padding (ids < 0).
// A half-wave (32 lanes x float4) per row at D = 128; rows of other widths by float lanes.
__global__ __launch_bounds__(256) void gather_padded_kernel(const float* __restrict__ shard,
                                                            int64_t n_rows, int dim,
                                                            const int32_t* __restrict__ ids,
                                                            int64_t n, float* __restrict__ out) {
  const bool vec = (dim & 3) == 0;
  const int lanes = vec ? (dim / 4 < 64 ? dim / 4 : 64) : (dim < 64 ? dim : 64);
  const int per_block = 256 / lanes;
  const int sub = threadIdx.x / lanes, l = threadIdx.x % lanes;
  if (sub >= per_block) return;
  for (int64_t i = blockIdx.x * (int64_t)per_block + sub; i < n;
       i += (int64_t)gridDim.x * per_block) {
    const int32_t r = ids[i];
    const bool ok = r >= 0 && r < n_rows;
    float* dst = out + i * dim;
    if (vec) {
      const float4* src = reinterpret_cast<const float4*>(shard + (ok ? (int64_t)r * dim : 0));
      for (int c = l; c < dim / 4; c += lanes)
        reinterpret_cast<float4*>(dst)[c] = ok ? src[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      for (int c = l; c < dim; c += lanes) dst[c] = ok ? shard[(int64_t)r * dim + c] : 0.f;
    }
  }
}

// The owner's side of the rows-ahead exchange: of the next step's requested slots (recv_ids, a
// [world, cap] block per requester), those whose row the step now finishing requested too
// (stamp[row] == pred: rows its apply changes) are listed per requester — late_rows[r·cap + k]
// = the local row, late_slot[r·cap + k] = its slot in r's block, late_cnt[r] = k's bound — and
// re-sent after that apply; every other slot's row is final when gathered a step early. Waves
// compact with a ballot per requester (a wave may straddle two blocks) and one atomic per
// (wave, requester), so the list order varies run to run, the rows it carries do not.
__global__ __launch_bounds__(256) void exchange_classify_kernel(
    const int32_t* __restrict__ recv_ids, int64_t n, int64_t cap, const int32_t* __restrict__ stamp,
    int64_t n_rows, int32_t pred, int32_t* __restrict__ late_rows, int32_t* __restrict__ late_slot,
    int32_t* __restrict__ late_cnt) {
  const int lane = threadIdx.x & 63;
  const int64_t n_pad = (n + 63) & ~int64_t(63);  // whole waves take every ballot
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_pad;
       i += (int64_t)gridDim.x * blockDim.x) {
    int32_t r = -1;
    if (i < n) r = recv_ids[i];
    const bool hit = r >= 0 && r < n_rows && stamp[r] == pred;
    const int64_t o = i / cap;
    uint64_t pending = __ballot(hit);
    while (pending) {
      const int leader = __ffsll((unsigned long long)pending) - 1;
      const int64_t ol = __shfl(o, leader);
      const bool mine = hit && o == ol;
      const uint64_t same = __ballot(mine);
      int32_t base = 0;
      if (lane == leader) base = atomicAdd(late_cnt + ol, __popcll(same));
      base = __shfl(base, leader);
      if (mine) {
        const int32_t k = base + __popcll(same & ((uint64_t(1) << lane) - 1));
        late_rows[ol * cap + k] = r;
        late_slot[ol * cap + k] = (int32_t)(i - ol * cap);
      }
      pending &= ~same;
    }
  }
}

// stamp[row] = seq for every requested row of a step (before the next step's classify)
__global__ __launch_bounds__(256) void exchange_mark_kernel(const int32_t* __restrict__ recv_ids,
                                                            int64_t n, int32_t* __restrict__ stamp,
                                                            int64_t n_rows, int32_t seq) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t r = recv_ids[i];
    if (r >= 0 && r < n_rows) stamp[r] = seq;
  }
}

// the requester's side: late row k of owner o (recv[o·cap_late + k]) overwrites its slot
// o·cap + slot[o·cap + k] of the rows gathered a step early; slot −1 is padding
__global__ __launch_bounds__(256) void exchange_scatter_late_kernel(
    const float* __restrict__ recv, const int32_t* __restrict__ slot, int world, int64_t cap,
    int64_t cap_late, int dim, float* __restrict__ rows) {
  const int lanes = 32, per_block = 256 / lanes;
  const int sub = threadIdx.x / lanes, l = threadIdx.x % lanes;
  const int64_t n = (int64_t)world * cap_late;
  for (int64_t e = blockIdx.x * (int64_t)per_block + sub; e < n;
       e += (int64_t)gridDim.x * per_block) {
    const int64_t o = e / cap_late, k = e - o * cap_late;
    const int32_t j = slot[o * cap + k];
    if (j < 0) continue;
    const float4* src = reinterpret_cast<const float4*>(recv + e * dim);
    float4* dst = reinterpret_cast<float4*>(rows + (o * cap + j) * dim);
    for (int c = l; c < dim / 4; c += lanes) dst[c] = src[c];
  }
}

}  // namespace rs

using namespace rs;

extern "C" int32_t rs_exchange_mark(const int32_t* recv_ids, int64_t n, int32_t* stamp,
                                    int64_t n_rows, int32_t seq, void* stream) {
  RS_CHECK_ARG(n >= 0 && n < (int64_t(1) << 31) && n_rows >= 0, "bad sizes");
  if (n == 0) return RS_OK;
  RS_CHECK_ARG(recv_ids && stamp, "null pointer");
  const int blocks = (int)std::min<int64_t>(ceil_div(n, 256), 2048);
  exchange_mark_kernel<<<blocks, 256, 0, as_stream(stream)>>>(recv_ids, n, stamp, n_rows, seq);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_exchange_classify(const int32_t* recv_ids, int32_t world, int64_t capacity,
                                        const int32_t* stamp, int64_t n_rows, int32_t pred_seq,
                                        int32_t* late_rows, int32_t* late_slot,
                                        int32_t* late_count, void* stream) {
  RS_CHECK_ARG(world >= 1 && world <= kMaxWorld && capacity > 0 && n_rows >= 0, "bad sizes");
  RS_CHECK_ARG((int64_t)world * capacity < (int64_t(1) << 31), "world x capacity out of range");
  RS_CHECK_ARG(recv_ids && stamp && late_rows && late_slot && late_count, "null pointer");
  hipStream_t st = as_stream(stream);
  const int64_t n = (int64_t)world * capacity;
  RS_CHECK_HIP(hipMemsetAsync(late_rows, 0xFF, (size_t)n * sizeof(int32_t), st));
  RS_CHECK_HIP(hipMemsetAsync(late_slot, 0xFF, (size_t)n * sizeof(int32_t), st));
  RS_CHECK_HIP(hipMemsetAsync(late_count, 0, (size_t)world * sizeof(int32_t), st));
  const int blocks = (int)std::min<int64_t>(ceil_div(n, 256), 2048);
  exchange_classify_kernel<<<blocks, 256, 0, st>>>(recv_ids, n, capacity, stamp, n_rows, pred_seq,
                                                   late_rows, late_slot, late_count);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_exchange_scatter_late(const float* recv_rows, const int32_t* recv_slot,
                                            int32_t world, int64_t capacity, int64_t late_capacity,
                                            int32_t dim, float* rows, void* stream) {
  RS_CHECK_ARG(world >= 1 && world <= kMaxWorld && capacity > 0, "bad sizes");
  RS_CHECK_ARG(late_capacity >= 0 && late_capacity <= capacity, "late capacity out of range");
  RS_CHECK_ARG(dim > 0 && (dim & 3) == 0, "dim must be a multiple of 4");
  if (late_capacity == 0) return RS_OK;
  RS_CHECK_ARG(recv_rows && recv_slot && rows, "null pointer");
  RS_CHECK_ARG(((reinterpret_cast<uintptr_t>(recv_rows) | reinterpret_cast<uintptr_t>(rows)) & 15) == 0,
               "rows must be 16-byte aligned");
  const int64_t n = (int64_t)world * late_capacity;
  const int blocks = (int)std::min<int64_t>(ceil_div(n, 8), 4096);
  exchange_scatter_late_kernel<<<blocks, 256, 0, as_stream(stream)>>>(recv_rows, recv_slot, world,
                                                                      capacity, late_capacity, dim,
                                                                      rows);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_exchange_pack(const uint32_t* uniq_keys, const int32_t* n_unique,
                                    const int32_t* owner_counts, int32_t world, int64_t shard_stride,
                                    int64_t capacity, const int32_t* inverse, int64_t n_ids,
                                    int32_t* send_ids, int32_t* slot_of_unique,
                                    int32_t* inverse_slot, int32_t* overflow, void* stream) {
  RS_CHECK_ARG(world >= 1 && world <= kMaxWorld, "world out of range");
  RS_CHECK_ARG(shard_stride > 0 && capacity > 0 && n_ids >= 0, "bad sizes");
  RS_CHECK_ARG((int64_t)world * capacity < (int64_t(1) << 31), "world x capacity out of range");
  RS_CHECK_ARG(send_ids && n_unique && owner_counts && overflow, "null pointer");
  hipStream_t st = as_stream(stream);
  RS_CHECK_HIP(hipMemsetAsync(send_ids, 0xFF, (size_t)world * capacity * sizeof(int32_t), st));
  if (n_ids == 0) return RS_OK;
  RS_CHECK_ARG(uniq_keys && inverse && slot_of_unique && inverse_slot, "null pointer");
  const int blocks = (int)std::min<int64_t>(ceil_div(n_ids, 256), 2048);
  exchange_slots_kernel<<<blocks, 256, 0, st>>>(uniq_keys, n_unique, owner_counts, world,
                                                shard_stride, capacity, n_ids, send_ids,
                                                slot_of_unique, overflow);
  RS_CHECK_LAUNCH();
  exchange_inverse_kernel<<<blocks, 256, 0, st>>>(inverse, slot_of_unique, n_ids, inverse_slot);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_exchange_excess(const int32_t* owner_counts, int32_t world, int64_t capacity,
                                      int64_t* excess, void* stream) {
  RS_CHECK_ARG(world >= 1 && world <= kMaxWorld && capacity >= 0, "bad sizes");
  RS_CHECK_ARG(owner_counts && excess, "null pointer");
  exchange_excess_kernel<<<1, 64, 0, as_stream(stream)>>>(owner_counts, world, capacity, excess);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_exchange_pack_spill(const uint32_t* uniq_keys, const int32_t* n_unique,
                                          const int32_t* owner_counts, int32_t world,
                                          int64_t shard_stride, int64_t capacity,
                                          int64_t spill_capacity, const int32_t* inverse,
                                          int64_t n_ids, int32_t* spill_ids,
                                          int32_t* slot_of_unique, int32_t* inverse_slot,
                                          int32_t* overflow, void* stream) {
  RS_CHECK_ARG(world >= 1 && world <= kMaxWorld, "world out of range");
  RS_CHECK_ARG(shard_stride > 0 && capacity > 0 && spill_capacity > 0 && n_ids >= 0, "bad sizes");
  RS_CHECK_ARG((int64_t)world * (capacity + spill_capacity) < (int64_t(1) << 31),
               "world x capacity out of range");
  RS_CHECK_ARG(spill_ids && n_unique && owner_counts, "null pointer");
  hipStream_t st = as_stream(stream);
  RS_CHECK_HIP(hipMemsetAsync(spill_ids, 0xFF, (size_t)world * spill_capacity * sizeof(int32_t), st));
  if (n_ids == 0) return RS_OK;
  RS_CHECK_ARG(uniq_keys && inverse && slot_of_unique && inverse_slot, "null pointer");
  const int blocks = (int)std::min<int64_t>(ceil_div(n_ids, 256), 2048);
  exchange_spill_slots_kernel<<<blocks, 256, 0, st>>>(uniq_keys, n_unique, owner_counts, world,
                                                      shard_stride, capacity, spill_capacity, n_ids,
                                                      spill_ids, slot_of_unique, overflow);
  RS_CHECK_LAUNCH();
  exchange_inverse_kernel<<<blocks, 256, 0, st>>>(inverse, slot_of_unique, n_ids, inverse_slot);
  RS_CHECK_LAUNCH();
  return RS_OK;
}

extern "C" int32_t rs_gather_rows_padded(const float* shard, int64_t n_rows, int32_t dim,
                                         const int32_t* ids, int64_t n, float* out, void* stream) {
  RS_CHECK_ARG(dim > 0 && n >= 0 && n_rows >= 0, "bad sizes");
  if (n == 0) return RS_OK;
  RS_CHECK_ARG(ids && out && (shard || n_rows == 0), "null pointer");
  RS_CHECK_ARG((dim & 3) != 0 || ((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(shard)) & 15) == 0,
               "rows of a multiple-of-4 width must be 16-byte aligned");
  hipStream_t st = as_stream(stream);
  const bool vec = (dim & 3) == 0;
  const int lanes = vec ? (dim / 4 < 64 ? dim / 4 : 64) : (dim < 64 ? dim : 64);
  const int64_t per_block = 256 / lanes;
  const int blocks = (int)std::min<int64_t>(ceil_div(n, per_block), 4096);
  gather_padded_kernel<<<blocks, 256, 0, st>>>(shard, n_rows, dim, ids, n, out);
  RS_CHECK_LAUNCH();
  return RS_OK;
}
