// Device-side synthetic generator: the GenModel rows of replicas [lo, hi) written straight
// into HBM (bench inputs; never part of a timed region). Row identities (src) are model
// coordinates so results can be cross-checked against host-generated snapshots:
//   data row src = i, expires src = U + i, deletes src = 2U + i,
//   node src = i * max_nodes + node slot, member src = i * member_universe + member index.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "engine.h"
#include "gen_model.h"
#include "partition.hip.h"

namespace cdb {
GenModel model_of(const cdb_gen_config& c);

namespace {

// (key, replica) entries with more children than this are filled by gen_big_kernel, one
// workgroup each (C5's hottest keys hold millions of children: one thread per key would
// serialise the whole generator behind them).
constexpr uint32_t kGenBig = 1024;

struct GenBig {  // one large (key, replica) entry
  uint64_t i, r, child0, key_row;
};

struct GenArgs {
  GenModel g;
  uint32_t lo, hi;
  uint32_t *ck, *cn, *cm;  // per key index counts
  unsigned long long* n_big;
  GenBig* big;             // capacity: the count kernel's n_big
  uint64_t* k[kKeyCols];
  uint64_t* nd[kNodeCols];
  uint64_t* mb[kMemberCols];
  uint32_t ks, cs;         // record strides (1: plain columns; the records layout, cdb_merge.h)
};
// field c of row i of a family (common.h row_field)
__device__ __forceinline__ uint64_t& gcell(uint64_t* const* col, uint32_t s, int c, uint64_t i) {
  return col[c][c ? i * s : i];
}

__global__ void gen_count_kernel(GenArgs a) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.g.universe;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t nk = 0, nn = 0, nm = 0, nbig = 0;
    const Hash128 h = gen_key_hash(i);
    if (gen_in_shard(a.g, h.h)) {
      for (uint32_t r = a.lo; r < a.hi; ++r) {
        if (gen_present(a.g, i, r)) {
          const GenKey k = gen_key(a.g, i, r);
          ++nk;
          if (k.tag == TAG_COUNTER) {
            nn += k.n_nodes;
            nbig += k.n_nodes > kGenBig;
          } else if (k.tag == TAG_SET || k.tag == TAG_DICT) {
            nm += k.n_members;
            nbig += k.n_members > kGenBig;
          }
        }
        nk += gen_has_expire(a.g, i, r);
        nk += gen_has_delete(a.g, i, r);
      }
    }
    a.ck[i] = nk;
    a.cn[i] = nn;
    a.cm[i] = nm;
    if (nbig) atomicAdd(a.n_big, (unsigned long long)nbig);
  }
}

__device__ __forceinline__ void gen_node_row(const GenArgs& a, const Hash128& h, const GenKey& k, uint64_t i,
                                             uint32_t r, uint32_t j, uint64_t pn, uint64_t v) {
  gcell(a.nd, a.cs, C_PKH, pn) = h.h;
  gcell(a.nd, a.cs, C_PKF, pn) = h.f;
  gcell(a.nd, a.cs, C_ID1, pn) = gen_node_id(a.g, k, j, r);
  gcell(a.nd, a.cs, C_ID2, pn) = v;
  gcell(a.nd, a.cs, C_T, pn) = gen_node_t(a.g, i, r, j);
  gcell(a.nd, a.cs, C_META, pn) = meta_pack(0, r, gen_node_src(a.g, i, j));
}
__device__ __forceinline__ void gen_member_row(const GenArgs& a, const Hash128& h, const GenKey& k, uint64_t i,
                                               uint32_t r, uint32_t j, uint64_t pm) {
  const uint64_t mi = gen_member_index(a.g, k, j);
  const Hash128 mh = gen_member_hash(mi);
  gcell(a.mb, a.cs, C_PKH, pm) = h.h;
  gcell(a.mb, a.cs, C_PKF, pm) = h.f;
  gcell(a.mb, a.cs, C_ID1, pm) = mh.h;
  gcell(a.mb, a.cs, C_ID2, pm) = mh.f;
  gcell(a.mb, a.cs, C_T, pm) = gen_member_t(a.g, i, r, j);
  gcell(a.mb, a.cs, C_META, pm) = meta_pack(gen_member_is_del(a.g, i, r, j) ? KIND_DEL : KIND_ADD, r, gen_member_src(a.g, i, mi));
}

__global__ void gen_fill_kernel(GenArgs a, const uint32_t* __restrict__ ok, const uint32_t* __restrict__ on,
                                const uint32_t* __restrict__ om) {
  const uint64_t U = a.g.universe;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < U; i += (uint64_t)gridDim.x * blockDim.x) {
    const Hash128 h = gen_key_hash(i);
    if (!gen_in_shard(a.g, h.h)) continue;
    uint64_t pk = ok[i], pn = on[i], pm = om[i];
    auto key_row = [&](uint64_t ct, uint64_t ut, uint64_t dt, uint64_t aux, uint64_t meta) {
      gcell(a.k, a.ks, K_KH, pk) = h.h;
      gcell(a.k, a.ks, K_KF, pk) = h.f;
      gcell(a.k, a.ks, K_CT, pk) = ct;
      gcell(a.k, a.ks, K_UT, pk) = ut;
      gcell(a.k, a.ks, K_DT, pk) = dt;
      gcell(a.k, a.ks, K_AUX, pk) = aux;
      gcell(a.k, a.ks, K_META, pk) = meta;
      ++pk;
    };
    for (uint32_t r = a.lo; r < a.hi; ++r) {
      if (gen_present(a.g, i, r)) {
        const GenKey k = gen_key(a.g, i, r);
        uint64_t aux = 0;
        const uint32_t nc = k.tag == TAG_COUNTER ? k.n_nodes : (k.tag == TAG_SET || k.tag == TAG_DICT) ? k.n_members : 0;
        if (nc > kGenBig) {  // filled by gen_big_kernel (a counter's total added there)
          const unsigned long long e = atomicAdd(a.n_big, 1ull);
          a.big[e] = GenBig{i, r, k.tag == TAG_COUNTER ? pn : pm, pk};
          (k.tag == TAG_COUNTER ? pn : pm) += nc;
        } else if (k.tag == TAG_COUNTER) {
          for (uint32_t j = 0; j < k.n_nodes; ++j, ++pn) {
            const uint64_t v = gen_node_v(a.g, i, r, j);
            aux += v;
            gen_node_row(a, h, k, i, r, j, pn, v);
          }
        } else if (k.tag == TAG_SET || k.tag == TAG_DICT) {
          for (uint32_t j = 0; j < k.n_members; ++j, ++pm) gen_member_row(a, h, k, i, r, j, pm);
        }
        key_row(k.ct, k.ut, k.dt, aux, meta_pack(k.tag, r, i));
      }
      if (gen_has_expire(a.g, i, r)) key_row(gen_time(a.g, i, r, 3), 0, 0, 0, meta_pack(TAG_EXPIRE, r, U + i));
      if (gen_has_delete(a.g, i, r)) key_row(gen_time(a.g, i, r, 4), 0, 0, 0, meta_pack(TAG_DELETE, r, 2 * U + i));
    }
  }
}

// One workgroup per large (key, replica) entry: its children, and a counter's total.
__global__ void __launch_bounds__(256) gen_big_kernel(GenArgs a, uint64_t n) {
  __shared__ unsigned long long part;
  for (uint64_t e = blockIdx.x; e < n; e += gridDim.x) {
    const GenBig B = a.big[e];
    const uint32_t r = (uint32_t)B.r;
    const Hash128 h = gen_key_hash(B.i);
    const GenKey k = gen_key(a.g, B.i, r);
    if (threadIdx.x == 0) part = 0;
    __syncthreads();
    unsigned long long sum = 0;
    if (k.tag == TAG_COUNTER) {
      for (uint32_t j = threadIdx.x; j < k.n_nodes; j += blockDim.x) {
        const uint64_t v = gen_node_v(a.g, B.i, r, j);
        sum += v;
        gen_node_row(a, h, k, B.i, r, j, B.child0 + j, v);
      }
      atomicAdd(&part, sum);
    } else {
      for (uint32_t j = threadIdx.x; j < k.n_members; j += blockDim.x) gen_member_row(a, h, k, B.i, r, j, B.child0 + j);
    }
    __syncthreads();
    if (threadIdx.x == 0 && k.tag == TAG_COUNTER) gcell(a.k, a.ks, K_AUX, B.key_row) += part;
    __syncthreads();
  }
}

}  // namespace
}  // namespace cdb

using namespace cdb;

extern "C" cdb_status cdb_gen_device(cdb_ctx* ctx, const cdb_gen_config* cfg, cdb_dev_input* in) {
  if (!ctx || !cfg || !in) return CDB_BAD_ARGUMENT;
  if (cfg->replica_hi > (uint32_t)kMaxPos || cfg->replica_lo >= cfg->replica_hi)
    return fail(ctx, CDB_BAD_ARGUMENT, "replica range");
  hipSetDevice(ctx->device);
  hipStream_t s = ctx->stream;
  GenArgs a;
  std::memset(&a, 0, sizeof a);
  a.g = model_of(*cfg);
  a.lo = cfg->replica_lo;
  a.hi = cfg->replica_hi;
  const uint64_t U = a.g.universe;
  uint32_t* cnt = nullptr;
  cdb_status st = hip_check(ctx, hipMalloc(&cnt, 6 * std::max<uint64_t>(U, 1) * sizeof(uint32_t)), "hipMalloc(gen)");
  if (st != CDB_OK) return st;
  a.ck = cnt;
  a.cn = cnt + U;
  a.cm = cnt + 2 * U;
  uint32_t *ok = cnt + 3 * U, *on = cnt + 4 * U, *om = cnt + 5 * U;
  uint64_t* tot = nullptr;
  st = hip_check(ctx, hipMalloc(&tot, 4 * sizeof(uint64_t)), "hipMalloc");
  if (st != CDB_OK) { hipFree(cnt); return st; }
  a.n_big = (unsigned long long*)(tot + 3);
  if ((st = hip_check(ctx, hipMemsetAsync(a.n_big, 0, 8, s), "memset")) != CDB_OK) { hipFree(cnt); hipFree(tot); return st; }
  const int grid = 4096, block = 256;
  gen_count_kernel<<<grid, block, 0, s>>>(a);
  // exclusive scans of the per-key counts
  auto scan = [&](const uint32_t* c, uint32_t* o, uint64_t* t) -> cdb_status {
    const uint64_t tiles = std::max<uint64_t>(1, (U + kScanTile - 1) / kScanTile);
    uint64_t* sums = nullptr;
    cdb_status s2 = hip_check(ctx, hipMalloc(&sums, tiles * 8), "hipMalloc");
    if (s2 != CDB_OK) return s2;
    scan_reduce_kernel<uint32_t><<<tiles, kScanThreads, 0, s>>>(c, U, sums);
    scan_sums_kernel<<<1, kScanThreads, 0, s>>>(sums, tiles, t);
    scan_apply_kernel<uint32_t, uint32_t><<<tiles, kScanThreads, 0, s>>>(c, U, sums, o, (uint32_t*)nullptr);
    s2 = hip_check(ctx, hipStreamSynchronize(s), "gen scan");
    hipFree(sums);
    return s2;
  };
  if ((st = scan(a.ck, ok, tot)) != CDB_OK || (st = scan(a.cn, on, tot + 1)) != CDB_OK ||
      (st = scan(a.cm, om, tot + 2)) != CDB_OK) {
    hipFree(cnt);
    hipFree(tot);
    return st;
  }
  uint64_t t[4];
  hipMemcpy(t, tot, sizeof t, hipMemcpyDeviceToHost);
  GenBig* big = nullptr;
  if (t[3] && (st = hip_check(ctx, hipMalloc(&big, t[3] * sizeof(GenBig)), "hipMalloc(gen big)")) != CDB_OK) {
    hipFree(cnt);
    hipFree(tot);
    return st;
  }
  a.big = big;
  if (t[0] >= (1ull << 32) || t[1] >= (1ull << 32) || t[2] >= (1ull << 32)) {
    hipFree(cnt);
    hipFree(tot);
    if (big) hipFree(big);
    return fail(ctx, CDB_BAD_ARGUMENT, "generated rows exceed 2^32 per family");
  }
  std::memset(in, 0, sizeof *in);
  const bool rec = cfg->flags & CDB_GEN_ROWS_RECORDS;
  auto alloc = [&](cdb_dev_rows* r, uint64_t rows, int nc) {
    return rec ? cdb_dev_rows_alloc_records(ctx, r, rows, nc) : cdb_dev_rows_alloc(ctx, r, rows, nc);
  };
  if ((st = alloc(&in->keys, t[0], kKeyCols)) != CDB_OK || (st = alloc(&in->nodes, t[1], kNodeCols)) != CDB_OK ||
      (st = alloc(&in->members, t[2], kMemberCols)) != CDB_OK) {
    hipFree(cnt);
    hipFree(tot);
    if (big) hipFree(big);
    return st;
  }
  a.ks = std::max<uint32_t>(in->keys.stride, 1);
  a.cs = std::max<uint32_t>(in->nodes.stride, 1);
  for (int c = 0; c < kKeyCols; ++c) a.k[c] = in->keys.col[c];
  for (int c = 0; c < kNodeCols; ++c) {
    a.nd[c] = in->nodes.col[c];
    a.mb[c] = in->members.col[c];
  }
  hipMemsetAsync(a.n_big, 0, 8, s);
  gen_fill_kernel<<<grid, block, 0, s>>>(a, ok, on, om);
  if (t[3]) gen_big_kernel<<<(uint32_t)std::min<uint64_t>(t[3], 4096), 256, 0, s>>>(a, t[3]);
  st = hip_check(ctx, hipStreamSynchronize(s), "gen fill");
  hipFree(cnt);
  hipFree(tot);
  if (big) hipFree(big);
  in->n_pos = cfg->replica_hi;
  return st;
}
