// rccl_stub.cpp -- test double of the five RCCL entry points libcmtverify
// resolves with dlopen (runtime.cpp load_rccl), for rehearsing the library's
// multi-rank code on a one-GPU box. Selected per context
// by CMTV_RCCL_LIB=<path to librccl_stub.so> together with CMTV_FORCE_RCCL=1
// over a repeated device ordinal. Test infrastructure: nothing in the product
// links or loads it by default.
//
// Semantics follow the NCCL API contract the library relies on:
//   ncclCommInitAll(comms, n, devlist)  one communicator per rank, rank i on
//                                       devlist[i];
//   ncclGroupStart / ncclGroupEnd       the ops between them are issued
//                                       together (one thread drives every rank);
//   ncclAllGather(send, recv, count, dtype, comm, stream)
//                                       recv[q*count ..] = rank q's send buffer
//                                       for every q, enqueued on `stream`;
//                                       in place when send == recv + rank*count.
// The gather is done with device-to-device copies ordered by HIP events: each
// rank's stream waits for every other rank's producers before reading their
// send buffers, and every rank's stream then waits for the readers of its own
// buffer (the stream ordering a real collective gives).
//
// CMTV_RCCL_STUB_FAIL_GROUP=k fails the communicator's k-th grouped call
// (ncclSystemError) with nothing copied; with CMTV_RCCL_STUB_PARTIAL=1 as
// well, rank 0's part of that call is left enqueued as a collective whose
// peers never arrive: its stream is held by a host callback until
// ncclCommAbort / ncclCommDestroy of the group (or a 10 s watchdog) releases
// it -- what a real group that fails after launching one rank's kernel does.
//
// Every call is appended to the file named by CMTV_RCCL_STUB_LOG (if set when
// the communicator was created), one line per event:
//   init n=<ranks> devs=<d0,d1,...> comm=<id>
//   allgather comm=<id> rank=<r> nranks=<n> count=<c> dtype=<t> inplace=<0|1>
//   destroy comm=<id> rank=<r>
// and rccl_stub_calls() reports the number of gathers executed.
#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

struct Group;
struct Comm {
  Group* g;
  int rank;
  int dev;
};
struct Group {
  int id;
  int n;
  int live;
  std::vector<int> devs;
  std::string log;  // CMTV_RCCL_STUB_LOG as it was at ncclCommInitAll
  int fail_at = 0;  // CMTV_RCCL_STUB_FAIL_GROUP: this group end (1-based) fails
  int ends = 0;
  bool partial = false;  // CMTV_RCCL_STUB_PARTIAL: ... after enqueueing rank 0
  struct Hold* hold = nullptr;  // rank 0's stuck collective, if any
};

// A stream held by a host callback until released (the stuck collective).
struct Hold {
  std::mutex m;
  std::condition_variable cv;
  bool released = false;
  void release() {
    std::lock_guard<std::mutex> lk(m);
    released = true;
    cv.notify_all();
  }
};

void hold_stream(void* arg) {
  auto* h = static_cast<Hold*>(arg);
  std::unique_lock<std::mutex> lk(h->m);
  h->cv.wait_for(lk, std::chrono::seconds(10), [h] { return h->released; });
}
struct Op {
  const void* send;
  void* recv;
  size_t count;
  int dtype;
  Comm* comm;
  hipStream_t stream;
};

std::mutex mu;
int next_id = 1;
long gathers = 0;
thread_local int depth = 0;
thread_local std::vector<Op> pending;

void log_line(const std::string& path, const std::string& s) {
  if (path.empty()) return;
  if (FILE* f = std::fopen(path.c_str(), "a")) {
    std::fputs(s.c_str(), f);
    std::fputc('\n', f);
    std::fclose(f);
  }
}

size_t dtype_size(int t) {
  switch (t) {
    case 0: case 1: return 1;          // int8, uint8
    case 2: case 3: case 7: return 4;  // int32, uint32, float32
    case 4: case 5: case 8: return 8;  // int64, uint64, float64
    case 6: return 2;                  // float16
    default: return 0;
  }
}

// Executes the gathers of one group call. Returns 0 or an ncclResult_t code.
int run_ops(std::vector<Op>& ops) {
  if (ops.empty()) return 0;
  // every op must belong to one communicator group and cover each rank once
  Group* g = ops[0].comm->g;
  std::vector<Op*> by_rank(g->n, nullptr);
  for (auto& o : ops) {
    if (o.comm->g != g || o.count != ops[0].count || o.dtype != ops[0].dtype) return 5;  // ncclInvalidUsage
    if (by_rank[o.comm->rank]) return 5;
    by_rank[o.comm->rank] = &o;
  }
  for (auto* o : by_rank)
    if (!o) return 5;  // a real all-gather would hang waiting for the missing rank
  const size_t bytes = ops[0].count * dtype_size(ops[0].dtype);
  if (!bytes) return 4;  // ncclInvalidArgument
  std::vector<hipEvent_t> ready(g->n), read(g->n);
  auto fail = [&](int rc) {
    for (auto e : ready) if (e) (void)hipEventDestroy(e);
    for (auto e : read) if (e) (void)hipEventDestroy(e);
    return rc;
  };
  for (int r = 0; r < g->n; r++) {
    const Op& o = *by_rank[r];
    if (hipSetDevice(o.comm->dev) != hipSuccess) return fail(1);
    if (hipEventCreateWithFlags(&ready[r], hipEventDisableTiming) != hipSuccess) return fail(1);
    if (hipEventCreateWithFlags(&read[r], hipEventDisableTiming) != hipSuccess) return fail(1);
    if (hipEventRecord(ready[r], o.stream) != hipSuccess) return fail(1);
  }
  for (int r = 0; r < g->n; r++) {
    const Op& o = *by_rank[r];
    (void)hipSetDevice(o.comm->dev);
    for (int q = 0; q < g->n; q++) {
      const Op& src = *by_rank[q];
      char* dst = static_cast<char*>(o.recv) + (size_t)q * bytes;
      if (q == r) {
        if (src.send != dst && hipMemcpyAsync(dst, src.send, bytes, hipMemcpyDeviceToDevice, o.stream) != hipSuccess)
          return fail(1);
        continue;
      }
      if (hipStreamWaitEvent(o.stream, ready[q], 0) != hipSuccess) return fail(1);
      if (hipMemcpyPeerAsync(dst, o.comm->dev, src.send, src.comm->dev, bytes, o.stream) != hipSuccess)
        return fail(1);
    }
    if (hipEventRecord(read[r], o.stream) != hipSuccess) return fail(1);
  }
  // a rank's buffer may be rewritten only after every other rank read it
  for (int q = 0; q < g->n; q++) {
    const Op& o = *by_rank[q];
    (void)hipSetDevice(o.comm->dev);
    for (int r = 0; r < g->n; r++)
      if (r != q && hipStreamWaitEvent(o.stream, read[r], 0) != hipSuccess) return fail(1);
  }
  {
    std::lock_guard<std::mutex> lk(mu);
    gathers++;
    for (int r = 0; r < g->n; r++) {
      const Op& o = *by_rank[r];
      const bool inplace = o.send == static_cast<const char*>(o.recv) + (size_t)r * bytes;
      log_line(g->log, "allgather comm=" + std::to_string(g->id) + " rank=" + std::to_string(r) +
               " nranks=" + std::to_string(g->n) + " count=" + std::to_string(o.count) +
               " dtype=" + std::to_string(o.dtype) + " inplace=" + std::to_string(inplace ? 1 : 0));
    }
  }
  // events are only referenced by enqueued waits, which hold their state
  return fail(0);
}

}  // namespace

extern "C" {

int ncclCommInitAll(void** comms, int ndev, const int* devlist) {
  if (!comms || ndev <= 0 || !devlist) return 4;
  std::lock_guard<std::mutex> lk(mu);
  const char* path = std::getenv("CMTV_RCCL_STUB_LOG");
  auto* g = new Group{next_id++, ndev, ndev, std::vector<int>(devlist, devlist + ndev), path ? path : ""};
  if (const char* f = std::getenv("CMTV_RCCL_STUB_FAIL_GROUP")) g->fail_at = std::atoi(f);
  if (const char* f = std::getenv("CMTV_RCCL_STUB_PARTIAL")) g->partial = f[0] == '1';
  std::string devs;
  for (int i = 0; i < ndev; i++) {
    comms[i] = new Comm{g, i, devlist[i]};
    devs += (i ? "," : "") + std::to_string(devlist[i]);
  }
  log_line(g->log, "init n=" + std::to_string(ndev) + " devs=" + devs + " comm=" + std::to_string(g->id));
  return 0;
}

static int release_comm(void* comm, const char* what) {
  if (!comm) return 4;
  auto* c = static_cast<Comm*>(comm);
  std::lock_guard<std::mutex> lk(mu);
  log_line(c->g->log, std::string(what) + " comm=" + std::to_string(c->g->id) + " rank=" + std::to_string(c->rank));
  Group* g = c->g;
  if (g->hold) g->hold->release();  // the stuck collective ends with its communicator
  delete c;
  // the Hold is leaked on purpose: a callback may still be returning from it
  if (--g->live == 0) delete g;
  return 0;
}

int ncclCommDestroy(void* comm) { return release_comm(comm, "destroy"); }

int ncclCommAbort(void* comm) { return release_comm(comm, "abort"); }

int ncclGroupStart() {
  depth++;
  return 0;
}

int ncclGroupEnd() {
  if (depth <= 0) return 5;
  if (--depth > 0) return 0;
  std::vector<Op> ops;
  ops.swap(pending);
  if (!ops.empty()) {
    // CMTV_RCCL_STUB_FAIL_GROUP=k: the communicator's k-th grouped call fails
    // as a broken node's would (ncclSystemError), with nothing copied
    Group* g = ops[0].comm->g;
    std::lock_guard<std::mutex> lk(mu);
    if (g->fail_at && ++g->ends == g->fail_at) {
      if (g->partial && !g->hold) {
        // rank 0's collective was launched before the group failed
        for (auto& o : ops)
          if (o.comm->rank == 0) {
            g->hold = new Hold();
            (void)hipSetDevice(o.comm->dev);
            if (hipLaunchHostFunc(o.stream, hold_stream, g->hold) != hipSuccess) g->hold->release();
            log_line(g->log, "partial rank=0 comm=" + std::to_string(g->id));
          }
      }
      log_line(g->log, "groupend failed comm=" + std::to_string(g->id));
      return 2;
    }
  }
  return run_ops(ops);
}

int ncclAllGather(const void* send, void* recv, size_t count, int dtype, void* comm, hipStream_t stream) {
  if (!send || !recv || !comm || !dtype_size(dtype)) return 4;
  pending.push_back(Op{send, recv, count, dtype, static_cast<Comm*>(comm), stream});
  if (depth > 0) return 0;
  // outside a group a single rank's call would block in real RCCL until its
  // peers join; one thread cannot do that, so a lone call of a multi-rank
  // communicator is a usage error
  std::vector<Op> ops;
  ops.swap(pending);
  return run_ops(ops);
}

long rccl_stub_calls(void) {
  std::lock_guard<std::mutex> lk(mu);
  return gathers;
}

}  // extern "C"
