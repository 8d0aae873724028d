// l7m_multi.cc — several GPUs from one process (include/l7match.h
// l7m_multi_*).
//
// The reference decides requests one at a time on each connection's
// goroutine (pkg/proxy/kafka.go:116-152) or Envoy worker
// (envoy/cilium_l7policy.cc:126-186); requests are independent, so a batch
// shards with no data-path exchange.  A device set holds one HIP stream and
// one counter buffer per device; an evaluation cuts the batch into
// contiguous byte-balanced shards (equal HBM traffic per GPU), enqueues each
// shard's kernels on its device (the rule set's program is replicated there
// by l7m_eval_device on first use), then sums the R + 2 per-rule counters
// with one ncclAllReduce over a single-process RCCL communicator
// (ncclCommInitAll) and reads device 0's copy.  RCCL is opened with dlopen on
// the first set of distinct devices (the process may already hold one, e.g.
// torch's), so the library has no link-time dependency on it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/l7match.h"

namespace {

struct Rccl {
  decltype(&ncclCommInitAll) init_all = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  bool ok = false;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    for (const char* name : {"librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so.1"}) {
      h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);  // an RCCL the process already holds
      if (h) break;
    }
    if (!h)
      for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
        h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
        if (h) break;
      }
    if (!h) return;
    r.init_all = reinterpret_cast<decltype(r.init_all)>(dlsym(h, "ncclCommInitAll"));
    r.destroy = reinterpret_cast<decltype(r.destroy)>(dlsym(h, "ncclCommDestroy"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(h, "ncclAllReduce"));
    r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
    r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
    r.ok = r.init_all && r.destroy && r.all_reduce && r.group_start && r.group_end;
  });
  return r;
}

// device buffer grown on demand (on the device current when called)
struct DBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool reserve(size_t want) {
    if (cap >= want) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t sz = want + want / 4;
    if (hipMalloc(&p, sz) != hipSuccess) {
      p = nullptr;
      return false;
    }
    cap = sz;
    return true;
  }
  void free() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct Dev {
  int id = 0;
  hipStream_t stream = nullptr;
  DBuf hits, arena, offs, ids, verd;  // counters; staging of the host-arena path
  std::vector<uint64_t> hhost;
  std::vector<uint64_t> roffs;        // host: the shard's offsets rebased to its first record
};

}  // namespace

struct l7m_multi {
  std::vector<Dev> devs;
  std::vector<ncclComm_t> comms;  // one per device when RCCL reduces the counters
  std::mutex mu;
};

namespace {

int set_dev(int id) { return hipSetDevice(id) == hipSuccess ? L7M_OK : L7M_EDEVICE; }

// Sum the devices' counter buffers (nctr u64 each, already written on their
// streams) into hits: one RCCL all-reduce, then device 0's copy; or, without
// RCCL, every device's copy summed on the host.
int reduce_counters(l7m_multi* m, size_t nctr, uint64_t* hits) {
  const size_t nd = m->devs.size();
  std::vector<uint64_t> sum(nctr, 0);
  if (!m->comms.empty()) {
    const Rccl& r = rccl();
    int rc = L7M_OK;
    if (r.group_start() != ncclSuccess) return L7M_EDEVICE;
    for (size_t d = 0; d < nd && rc == L7M_OK; ++d) {
      if (set_dev(m->devs[d].id) != L7M_OK ||
          r.all_reduce(m->devs[d].hits.p, m->devs[d].hits.p, nctr, ncclUint64, ncclSum, m->comms[d],
                       m->devs[d].stream) != ncclSuccess)
        rc = L7M_EDEVICE;
    }
    if (r.group_end() != ncclSuccess) rc = L7M_EDEVICE;
    if (rc != L7M_OK) return rc;
    Dev& d0 = m->devs[0];
    if (set_dev(d0.id) != L7M_OK ||
        hipMemcpyAsync(sum.data(), d0.hits.p, nctr * 8, hipMemcpyDeviceToHost, d0.stream) != hipSuccess ||
        hipStreamSynchronize(d0.stream) != hipSuccess)
      return L7M_EDEVICE;
    for (size_t d = 1; d < nd; ++d)  // the other devices' all-reduces have completed too
      if (set_dev(m->devs[d].id) != L7M_OK || hipStreamSynchronize(m->devs[d].stream) != hipSuccess)
        return L7M_EDEVICE;
  } else {
    for (size_t d = 0; d < nd; ++d) {
      Dev& x = m->devs[d];
      x.hhost.resize(nctr);
      if (set_dev(x.id) != L7M_OK ||
          hipMemcpyAsync(x.hhost.data(), x.hits.p, nctr * 8, hipMemcpyDeviceToHost, x.stream) != hipSuccess ||
          hipStreamSynchronize(x.stream) != hipSuccess)
        return L7M_EDEVICE;
      for (size_t i = 0; i < nctr; ++i) sum[i] += x.hhost[i];
    }
  }
  for (size_t i = 0; i < nctr; ++i) hits[i] += sum[i];
  return L7M_OK;
}

}  // namespace

extern "C" {

int l7m_multi_create(const int* devices, uint32_t n_devices, l7m_multi** out) {
  if (!devices || !n_devices || !out) return L7M_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return L7M_EDEVICE;
  for (uint32_t k = 0; k < n_devices; ++k)
    if (devices[k] < 0 || devices[k] >= ndev) return L7M_EINVAL;
  int cur = 0;
  (void)hipGetDevice(&cur);
  auto* m = new (std::nothrow) l7m_multi();
  if (!m) return L7M_ENOMEM;
  m->devs.resize(n_devices);
  int rc = L7M_OK;
  for (uint32_t k = 0; k < n_devices && rc == L7M_OK; ++k) {
    Dev& d = m->devs[k];
    d.id = devices[k];
    if (set_dev(d.id) != L7M_OK || hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking) != hipSuccess)
      rc = L7M_EDEVICE;
  }
  std::vector<int> ids(devices, devices + n_devices);
  std::sort(ids.begin(), ids.end());
  const bool distinct = std::adjacent_find(ids.begin(), ids.end()) == ids.end();
  const char* no = std::getenv("L7M_MULTI_NO_RCCL");
  if (rc == L7M_OK && n_devices > 1 && distinct && !(no && no[0] == '1') && rccl().ok) {
    m->comms.resize(n_devices);
    if (rccl().init_all(m->comms.data(), static_cast<int>(n_devices), devices) != ncclSuccess) rc = L7M_EDEVICE;
  }
  (void)hipSetDevice(cur);
  if (rc != L7M_OK) {
    m->comms.clear();
    l7m_multi_destroy(m);
    return rc;
  }
  *out = m;
  return L7M_OK;
}

void l7m_multi_destroy(l7m_multi* m) {
  if (!m) return;
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (ncclComm_t c : m->comms)
    if (c) (void)rccl().destroy(c);
  for (Dev& d : m->devs) {
    if (hipSetDevice(d.id) != hipSuccess) continue;
    if (d.stream) (void)hipStreamSynchronize(d.stream);
    d.hits.free();
    d.arena.free();
    d.offs.free();
    d.ids.free();
    d.verd.free();
    if (d.stream) (void)hipStreamDestroy(d.stream);
  }
  (void)hipSetDevice(cur);
  delete m;
}

int l7m_multi_uses_rccl(const l7m_multi* m) { return m && !m->comms.empty() ? 1 : 0; }

int l7m_shard_bounds(const uint64_t* offs, size_t n, size_t arena_bytes, uint32_t parts, uint64_t* bounds) {
  if (!bounds || !parts || (n && !offs)) return L7M_EINVAL;
  for (size_t i = 1; i < n; ++i)
    if (offs[i] < offs[i - 1]) return L7M_EINVAL;
  if (n && offs[n - 1] >= arena_bytes) return L7M_EINVAL;
  bounds[0] = 0;
  for (uint32_t r = 1; r < parts; ++r) {
    if (!n) {
      bounds[r] = 0;
      continue;
    }
    // the first record starting at or past r / parts of the bytes from the first record on
    const unsigned __int128 total = arena_bytes - offs[0];
    const uint64_t target = offs[0] + static_cast<uint64_t>(total * r / parts);
    const uint64_t cut = static_cast<uint64_t>(std::lower_bound(offs, offs + n, target) - offs);
    bounds[r] = std::max<uint64_t>(cut, bounds[r - 1]);
  }
  bounds[parts] = n;
  return L7M_OK;
}

int l7m_multi_eval_device(l7m_multi* m, const l7m_ruleset* rs, const l7m_shard* shards, uint64_t* hits,
                          uint32_t flags) {
  if (!m || !rs || !shards) return L7M_EINVAL;
  l7m_ruleset_info info;
  l7m_ruleset_get_info(rs, &info);
  const size_t nctr = info.n_counters;
  std::lock_guard<std::mutex> g(m->mu);
  int cur = 0;
  (void)hipGetDevice(&cur);
  int rc = L7M_OK;
  for (size_t k = 0; k < m->devs.size() && rc == L7M_OK; ++k) {
    Dev& d = m->devs[k];
    const l7m_shard& s = shards[k];
    rc = set_dev(d.id);
    if (rc == L7M_OK && hits && (!d.hits.reserve(nctr * 8) ||
                                 hipMemsetAsync(d.hits.p, 0, nctr * 8, d.stream) != hipSuccess))
      rc = L7M_ENOMEM;
    if (rc == L7M_OK && s.n)
      rc = s.src_identities
               ? l7m_eval_device_ids(rs, s.arena, s.arena_bytes, s.rec_offsets, s.n, s.src_identities, s.verdicts,
                                     hits ? d.hits.p : nullptr, d.stream, flags)
               : l7m_eval_device(rs, s.arena, s.arena_bytes, s.rec_offsets, s.n, s.verdicts,
                                 hits ? d.hits.p : nullptr, d.stream, flags);
  }
  if (rc == L7M_OK && hits) rc = reduce_counters(m, nctr, hits);
  for (Dev& d : m->devs)
    if (hipSetDevice(d.id) != hipSuccess || hipStreamSynchronize(d.stream) != hipSuccess) rc = L7M_EDEVICE;
  (void)hipSetDevice(cur);
  return rc;
}

int l7m_multi_eval(l7m_multi* m, const l7m_ruleset* rs, const uint8_t* arena, size_t arena_bytes,
                   const uint64_t* offsets, size_t n, const uint32_t* ids, int32_t* verdicts, uint64_t* hits,
                   uint32_t flags) {
  if (!m || !rs || (n && (!arena || !offsets || !verdicts))) return L7M_EINVAL;
  const size_t nd = m->devs.size();
  std::vector<uint64_t> b(nd + 1);
  int rc = l7m_shard_bounds(offsets, n, arena_bytes, static_cast<uint32_t>(nd), b.data());
  if (rc != L7M_OK) return rc;
  l7m_ruleset_info info;
  l7m_ruleset_get_info(rs, &info);
  const size_t nctr = info.n_counters;
  std::lock_guard<std::mutex> g(m->mu);
  int cur = 0;
  (void)hipGetDevice(&cur);
  // one host thread per device: pageable H2D copies would otherwise serialise the devices
  std::vector<int> rcs(nd, L7M_OK);
  auto work = [&](size_t k) {
    Dev& d = m->devs[k];
    int& r = rcs[k];
    r = set_dev(d.id);
    const size_t lo = b[k], hi = b[k + 1], cnt = hi - lo;
    const uint64_t a = cnt ? offsets[lo] : 0, e = hi < n ? offsets[hi] : arena_bytes;
    const size_t bytes = static_cast<size_t>(e - a), padded = (bytes + 64 + 15) & ~size_t(15);
    if (r == L7M_OK && hits && (!d.hits.reserve(nctr * 8) ||
                                hipMemsetAsync(d.hits.p, 0, nctr * 8, d.stream) != hipSuccess))
      r = L7M_ENOMEM;
    if (r != L7M_OK || !cnt) return;
    d.roffs.resize(cnt);
    for (size_t i = 0; i < cnt; ++i) d.roffs[i] = offsets[lo + i] - a;
    if (!d.arena.reserve(padded) || !d.offs.reserve(cnt * 8) || !d.verd.reserve(cnt * 4) ||
        (ids && !d.ids.reserve(cnt * 4))) {
      r = L7M_ENOMEM;
      return;
    }
    auto* da = static_cast<uint8_t*>(d.arena.p);
    if (hipMemsetAsync(da + bytes, 0, padded - bytes, d.stream) != hipSuccess ||
        hipMemcpyAsync(da, arena + a, bytes, hipMemcpyHostToDevice, d.stream) != hipSuccess ||
        hipMemcpyAsync(d.offs.p, d.roffs.data(), cnt * 8, hipMemcpyHostToDevice, d.stream) != hipSuccess ||
        (ids && hipMemcpyAsync(d.ids.p, ids + lo, cnt * 4, hipMemcpyHostToDevice, d.stream) != hipSuccess)) {
      r = L7M_EDEVICE;
      return;
    }
    r = ids ? l7m_eval_device_ids(rs, da, bytes, d.offs.p, cnt, d.ids.p, d.verd.p, hits ? d.hits.p : nullptr,
                                  d.stream, flags)
            : l7m_eval_device(rs, da, bytes, d.offs.p, cnt, d.verd.p, hits ? d.hits.p : nullptr, d.stream, flags);
    if (r == L7M_OK &&
        (hipMemcpyAsync(verdicts + lo, d.verd.p, cnt * 4, hipMemcpyDeviceToHost, d.stream) != hipSuccess ||
         hipStreamSynchronize(d.stream) != hipSuccess))
      r = L7M_EDEVICE;
  };
  if (nd == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (size_t k = 0; k < nd; ++k) th.emplace_back(work, k);
    for (auto& t : th) t.join();
  }
  for (int r : rcs)
    if (r != L7M_OK && rc == L7M_OK) rc = r;
  if (rc == L7M_OK && hits) rc = reduce_counters(m, nctr, hits);
  for (Dev& d : m->devs)
    if (hipSetDevice(d.id) != hipSuccess || hipStreamSynchronize(d.stream) != hipSuccess) rc = L7M_EDEVICE;
  (void)hipSetDevice(cur);
  return rc;
}

}  // extern "C"
