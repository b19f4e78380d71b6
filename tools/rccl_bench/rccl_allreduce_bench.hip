// RCCL collective micro-benchmark for one MI355X node -- the fabric-validation role of the
// OSU micro-benchmarks the reference builds into its container
// (/root/reference/install-scripts/install_osu_bench.sh:13-17,
//  /root/reference/install-scripts/tf-hvd-gcc-ompi-ucx-mlnx-osu.def:25-26,61).
//
// One process per GPU, forked BEFORE any HIP call (no MPI, no exec after GPU init); rank 0's
// ncclUniqueId reaches the other ranks through pipes. For every message size it reports the
// max-over-ranks time, algorithm bandwidth and bus bandwidth (the number comparable to the
// per-link xGMI rate: allreduce busbw = algbw * 2(n-1)/n) and checks the result.
//
//   rccl_allreduce_bench [-n ranks] [-b min_bytes] [-e max_bytes] [-f factor] [-d float|bf16|half]
//                        [-t allreduce|reduce_scatter|allgather|broadcast|sendrecv]
//                        [-w warmup] [-i iters] [-o sum|avg] [-p 0|1 in-place] [-j json_path]
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CHECK_HIP(x)                                                                  \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      _exit(3);                                                                       \
    }                                                                                 \
  } while (0)
#define CHECK_NCCL(x)                                                                 \
  do {                                                                                \
    ncclResult_t r_ = (x);                                                            \
    if (r_ != ncclSuccess) {                                                          \
      fprintf(stderr, "RCCL error %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, __LINE__); \
      _exit(4);                                                                       \
    }                                                                                 \
  } while (0)

struct Opts {
  int nranks = 1;
  size_t minb = 8, maxb = (size_t)1 << 30;
  int factor = 2;
  std::string dtype = "float", test = "allreduce", op = "sum", json;
  int warmup = 5, iters = 20, inplace = 1;
};

static ncclDataType_t nccl_type(const std::string& d, int* esz) {
  if (d == "bf16") { *esz = 2; return ncclBfloat16; }
  if (d == "half") { *esz = 2; return ncclFloat16; }
  *esz = 4;
  return ncclFloat32;
}

// fill with a per-rank constant (exactly representable: ranks <= 8, sums <= 36)
__global__ void fill_kernel(float* p, size_t n, float v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}
__global__ void fill16_kernel(uint16_t* p, size_t n, uint16_t bits) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = bits;
}
// count elements != expect
__global__ void check_kernel(const void* p, size_t n, int esz, int is_bf16, float expect, unsigned* bad) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned local = 0;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float v;
    if (esz == 4) {
      v = reinterpret_cast<const float*>(p)[i];
    } else {
      uint16_t b = reinterpret_cast<const uint16_t*>(p)[i];
      if (is_bf16) {
        v = __uint_as_float((uint32_t)b << 16);
      } else {
        v = __half2float(*reinterpret_cast<const __half*>(&b));
      }
    }
    if (fabsf(v - expect) > 1e-3f * fabsf(expect) + 1e-6f) ++local;
  }
  if (local) atomicAdd(bad, local);
}

static uint16_t to_bits16(float v, bool bf16) {
  if (bf16) {
    uint32_t u;
    memcpy(&u, &v, 4);
    return (uint16_t)(u >> 16);  // exact for the small integers used here
  }
  __half h = __float2half(v);
  uint16_t b;
  memcpy(&b, &h, 2);
  return b;
}

static int run_rank(const Opts& o, int rank, ncclUniqueId uid) {
  CHECK_HIP(hipSetDevice(rank));
  ncclComm_t comm;
  CHECK_NCCL(ncclCommInitRank(&comm, o.nranks, uid, rank));
  hipStream_t st;
  CHECK_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int esz;
  const ncclDataType_t dt = nccl_type(o.dtype, &esz);
  const bool bf16 = o.dtype == "bf16";
  const ncclRedOp_t op = o.op == "avg" ? ncclAvg : ncclSum;
  const int n = o.nranks;
  void *sbuf = nullptr, *rbuf = nullptr;
  const size_t maxb = o.maxb;
  CHECK_HIP(hipMalloc(&sbuf, maxb));
  CHECK_HIP(hipMalloc(&rbuf, maxb * (o.test == "allgather" ? (size_t)n : 1)));
  unsigned* bad;
  CHECK_HIP(hipMalloc(&bad, sizeof(unsigned)));
  double* tdev;
  CHECK_HIP(hipMalloc(&tdev, sizeof(double)));
  hipEvent_t e0, e1;
  CHECK_HIP(hipEventCreate(&e0));
  CHECK_HIP(hipEventCreate(&e1));
  FILE* jf = nullptr;
  if (rank == 0) {
    printf("# RCCL %s  ranks=%d dtype=%s op=%s inplace=%d warmup=%d iters=%d\n", o.test.c_str(), n, o.dtype.c_str(),
           o.op.c_str(), o.inplace, o.warmup, o.iters);
    printf("%12s %12s %10s %10s %10s %6s\n", "bytes", "count", "time_us", "algbw_GB/s", "busbw_GB/s", "wrong");
    if (!o.json.empty()) {
      jf = fopen(o.json.c_str(), "w");
      if (jf) fprintf(jf, "{\"test\": \"%s\", \"ranks\": %d, \"dtype\": \"%s\", \"rows\": [", o.test.c_str(), n,
                      o.dtype.c_str());
    }
  }
  bool first = true;
  int rc = 0;
  for (size_t bytes = o.minb; bytes <= maxb; bytes *= (size_t)o.factor) {
    size_t count = bytes / esz;
    if (o.test == "reduce_scatter" || o.test == "allgather") count = count / n;
    if (count == 0) continue;
    const size_t nelem_send = (o.test == "reduce_scatter") ? count * n : count;
    const float v = (float)(rank + 1);
    if (esz == 4)
      hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, st, (float*)sbuf, nelem_send, v);
    else
      hipLaunchKernelGGL(fill16_kernel, dim3(1024), dim3(256), 0, st, (uint16_t*)sbuf, nelem_send, to_bits16(v, bf16));
    void* dst = (o.inplace && o.test == "allreduce") ? sbuf : rbuf;
    auto issue = [&]() {
      if (o.test == "allreduce") {
        CHECK_NCCL(ncclAllReduce(sbuf, dst, count, dt, op, comm, st));
      } else if (o.test == "reduce_scatter") {
        CHECK_NCCL(ncclReduceScatter(sbuf, rbuf, count, dt, op, comm, st));
      } else if (o.test == "allgather") {
        CHECK_NCCL(ncclAllGather(sbuf, rbuf, count, dt, comm, st));
      } else if (o.test == "broadcast") {
        CHECK_NCCL(ncclBroadcast(sbuf, rbuf, count, dt, 0, comm, st));
      } else {  // sendrecv around the ring
        CHECK_NCCL(ncclGroupStart());
        CHECK_NCCL(ncclSend(sbuf, count, dt, (rank + 1) % n, comm, st));
        CHECK_NCCL(ncclRecv(rbuf, count, dt, (rank + n - 1) % n, comm, st));
        CHECK_NCCL(ncclGroupEnd());
      }
    };
    // correctness pass (the in-place allreduce re-fills before timing)
    issue();
    float expect;
    const void* chk = dst;
    size_t nchk = count;
    if (o.test == "allreduce" || o.test == "reduce_scatter") {
      expect = (float)(n * (n + 1) / 2);
      if (o.op == "avg") expect /= (float)n;
      chk = (o.test == "allreduce") ? dst : rbuf;
    } else if (o.test == "allgather") {
      expect = 1.0f;  // checked on the first rank's slice below
      nchk = count;
    } else if (o.test == "broadcast") {
      expect = 1.0f;
    } else {
      expect = (float)(((rank + n - 1) % n) + 1);
    }
    CHECK_HIP(hipMemsetAsync(bad, 0, sizeof(unsigned), st));
    hipLaunchKernelGGL(check_kernel, dim3(1024), dim3(256), 0, st, chk, nchk, esz, bf16 ? 1 : 0, expect, bad);
    unsigned nbad = 0;
    CHECK_HIP(hipMemcpyAsync(&nbad, bad, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    CHECK_HIP(hipStreamSynchronize(st));
    if (nbad) rc = 5;
    for (int i = 0; i < o.warmup; ++i) issue();
    CHECK_HIP(hipEventRecord(e0, st));
    for (int i = 0; i < o.iters; ++i) issue();
    CHECK_HIP(hipEventRecord(e1, st));
    CHECK_HIP(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK_HIP(hipEventElapsedTime(&ms, e0, e1));
    double us = 1000.0 * ms / o.iters;
    CHECK_HIP(hipMemcpyAsync(tdev, &us, sizeof(double), hipMemcpyHostToDevice, st));
    CHECK_NCCL(ncclAllReduce(tdev, tdev, 1, ncclFloat64, ncclMax, comm, st));
    CHECK_HIP(hipMemcpyAsync(&us, tdev, sizeof(double), hipMemcpyDeviceToHost, st));
    CHECK_HIP(hipStreamSynchronize(st));
    const double data = (double)count * esz * ((o.test == "reduce_scatter" || o.test == "allgather") ? n : 1);
    const double algbw = data / us / 1e3;
    double f = 1.0;
    if (o.test == "allreduce") f = 2.0 * (n - 1) / n;
    else if (o.test == "reduce_scatter" || o.test == "allgather") f = (double)(n - 1) / n;
    const double busbw = algbw * f;
    if (rank == 0) {
      printf("%12zu %12zu %10.2f %10.2f %10.2f %6u\n", (size_t)data, count, us, algbw, busbw, nbad);
      fflush(stdout);
      if (jf) {
        fprintf(jf, "%s{\"bytes\": %zu, \"time_us\": %.3f, \"algbw\": %.3f, \"busbw\": %.3f, \"wrong\": %u}",
                first ? "" : ", ", (size_t)data, us, algbw, busbw, nbad);
        first = false;
      }
    }
  }
  if (jf) {
    fprintf(jf, "]}\n");
    fclose(jf);
  }
  CHECK_NCCL(ncclCommDestroy(comm));
  CHECK_HIP(hipFree(sbuf));
  CHECK_HIP(hipFree(rbuf));
  CHECK_HIP(hipFree(bad));
  CHECK_HIP(hipFree(tdev));
  return rc;
}

static size_t parse_size(const char* s) {
  char* end;
  double v = strtod(s, &end);
  switch (*end) {
    case 'K': case 'k': v *= 1024; break;
    case 'M': case 'm': v *= 1024 * 1024; break;
    case 'G': case 'g': v *= 1024.0 * 1024 * 1024; break;
    default: break;
  }
  return (size_t)v;
}

int main(int argc, char** argv) {
  Opts o;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> const char* {
      if (i + 1 >= argc) { fprintf(stderr, "missing value for %s\n", a.c_str()); exit(2); }
      return argv[++i];
    };
    if (a == "-n") o.nranks = atoi(next());
    else if (a == "-b") o.minb = parse_size(next());
    else if (a == "-e") o.maxb = parse_size(next());
    else if (a == "-f") o.factor = atoi(next());
    else if (a == "-d") o.dtype = next();
    else if (a == "-t") o.test = next();
    else if (a == "-w") o.warmup = atoi(next());
    else if (a == "-i") o.iters = atoi(next());
    else if (a == "-o") o.op = next();
    else if (a == "-p") o.inplace = atoi(next());
    else if (a == "-j") o.json = next();
    else {
      fprintf(stderr, "usage: %s [-n ranks] [-b min] [-e max] [-f factor] [-d float|bf16|half] "
              "[-t allreduce|reduce_scatter|allgather|broadcast|sendrecv] [-w N] [-i N] [-o sum|avg] [-p 0|1] [-j out.json]\n",
              argv[0]);
      return 2;
    }
  }
  if (o.nranks < 1 || o.nranks > 64 || o.factor < 2 || o.minb < 1 || o.maxb < o.minb) {
    fprintf(stderr, "bad arguments\n");
    return 2;
  }
  // pipes carry the unique id from rank 0 to the others; fork before any HIP/RCCL call
  std::vector<int> rd(o.nranks, -1), wr(o.nranks, -1);
  for (int r = 1; r < o.nranks; ++r) {
    int fd[2];
    if (pipe(fd) != 0) { perror("pipe"); return 1; }
    rd[r] = fd[0];
    wr[r] = fd[1];
  }
  std::vector<pid_t> kids;
  for (int r = 0; r < o.nranks; ++r) {
    pid_t pid = fork();
    if (pid < 0) { perror("fork"); return 1; }
    if (pid == 0) {
      ncclUniqueId uid;
      if (r == 0) {
        CHECK_NCCL(ncclGetUniqueId(&uid));
        for (int k = 1; k < o.nranks; ++k)
          if (write(wr[k], &uid, sizeof(uid)) != (ssize_t)sizeof(uid)) _exit(6);
      } else {
        size_t got = 0;
        while (got < sizeof(uid)) {
          ssize_t m = read(rd[r], reinterpret_cast<char*>(&uid) + got, sizeof(uid) - got);
          if (m <= 0) _exit(6);
          got += (size_t)m;
        }
      }
      _exit(run_rank(o, r, uid));
    }
    kids.push_back(pid);
  }
  int worst = 0;
  for (pid_t k : kids) {
    int status = 0;
    waitpid(k, &status, 0);
    int code = WIFEXITED(status) ? WEXITSTATUS(status) : 128 + (WIFSIGNALED(status) ? WTERMSIG(status) : 0);
    if (code > worst) worst = code;
  }
  return worst;
}
