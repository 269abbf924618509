// The machine's floor under the GAE scan: rocprofv3 / HIP-event durations of
//   empty      an empty kernel at gae_pipe_kernel's grid (4096 envs: 256 blocks x 256 threads)
//   ld1st1     one f32 load + one f32 store per thread at that grid
//   scanbytes  the scan's exact memory traffic at that grid with no chain: every thread issues the
//              8 slots' V, V', reward (f64), terminated, done loads up front (the same addresses
//              gae_pipe_kernel reads, 25 B per (env, step)) and stores adv / vtarget for them
//   scanbytes_wide  the same bytes over 4x as many, 4x smaller blocks (EB = 4 envs per block)
// at T = 128 and N = 4096 (the headline) and N = 16384 / 65536 (the scan sweep).  Not part of the
// engine: a stand-alone measurement, built by tools/gpu.sh (hipcc) on the box.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ void empty_kernel() {}

__global__ void ld1st1_kernel(const float *__restrict__ in, float *__restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  out[i] = in[i] + 1.f;
}

// EB envs per block, 16 time rows per chunk, KMAX chunks: thread (tt, c) -> rows T-1-(16k+tt)
template <int EB, int KMAX>
__global__ __launch_bounds__(EB * 16) void scanbytes_kernel(const float *__restrict__ v,
                                                            const float *__restrict__ vn,
                                                            const double *__restrict__ r,
                                                            const uint8_t *__restrict__ term,
                                                            const uint8_t *__restrict__ done, int n,
                                                            int t_len, float *__restrict__ adv,
                                                            float *__restrict__ vt) {
  const int tid = threadIdx.x, c = tid % EB, tt = tid / EB;
  const int env = blockIdx.x * EB + c;
  float lv[KMAX], lvn[KMAX];
  double lr[KMAX];
  uint8_t lt[KMAX], ld[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    const int t = t_len - 1 - (16 * k + tt);
    const int64_t idx = static_cast<int64_t>(t >= 0 ? t : 0) * n + env;
    lv[k] = v[idx];
    lvn[k] = vn[idx];
    lr[k] = r[idx];
    lt[k] = term[idx];
    ld[k] = done[idx];
  }
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    const int t = t_len - 1 - (16 * k + tt);
    if (t < 0) continue;
    const int64_t idx = static_cast<int64_t>(t) * n + env;
    const float a = static_cast<float>(lr[k]) + lvn[k] * (lt[k] ? 0.f : 0.99f) - lv[k] + (ld[k] ? 1.f : 0.f);
    adv[idx] = a;
    vt[idx] = a + lv[k];
  }
}

// the GAE recurrence's dependent chain alone: STEPS x (v_mul_f64, v_add_f64) on registers, one
// wave per block, 16 active lanes -- its duration minus the empty kernel's is the chain latency
template <int STEPS>
__global__ __launch_bounds__(64) void chain_kernel(const double *__restrict__ dq, double *__restrict__ out) {
  const int lane = threadIdx.x;
  if (lane >= 16) return;
  double d[16], q[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    d[j] = dq[2 * j];
    q[j] = dq[2 * j + 1];
  }
  double prev = 0.0;
  for (int s = 0; s < STEPS / 16; ++s) {
#pragma unroll
    for (int j = 0; j < 16; ++j) prev = d[j] + prev * q[j];
  }
  out[blockIdx.x * 16 + lane] = prev;
}

struct Bufs {
  float *v, *vn, *adv, *vt, *in, *out;
  double *r;
  uint8_t *term, *done;
};

// mean per-launch duration from an event pair on each dispatch packet (hipExtLaunchKernelGGL: the
// engine's own method, timing.h), after 20 warm-up launches
template <class K, class... Args>
static double time_us(K kernel, int grid, int block, int reps, Args... args) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 20; ++i) hipExtLaunchKernelGGL(kernel, dim3(grid), dim3(block), 0, 0, nullptr, nullptr, 0, args...);
  CK(hipDeviceSynchronize());
  double total = 0.0;
  for (int i = 0; i < reps; ++i) {
    hipExtLaunchKernelGGL(kernel, dim3(grid), dim3(block), 0, 0, a, b, 0, args...);
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    total += ms;
  }
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 1e3 * total / reps;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  const int T = 128;
  const int64_t nmax = 65536;
  Bufs B{};
  const size_t cells = static_cast<size_t>(T) * nmax;
  CK(hipMalloc(&B.v, cells * 4));
  CK(hipMalloc(&B.vn, cells * 4));
  CK(hipMalloc(&B.adv, cells * 4));
  CK(hipMalloc(&B.vt, cells * 4));
  CK(hipMalloc(&B.r, cells * 8));
  CK(hipMalloc(&B.term, cells));
  CK(hipMalloc(&B.done, cells));
  CK(hipMalloc(&B.in, 1 << 22));
  CK(hipMalloc(&B.out, 1 << 22));
  CK(hipMemset(B.v, 0, cells * 4));
  CK(hipMemset(B.vn, 0, cells * 4));
  CK(hipMemset(B.r, 0, cells * 8));
  CK(hipMemset(B.term, 0, cells));
  CK(hipMemset(B.done, 0, cells));
  CK(hipMemset(B.in, 0, 1 << 22));
  printf("[\n");
  bool first = true;
  auto emit = [&](const char *name, int n, int grid, int block, double us, double bytes) {
    printf("%s{\"kernel\": \"%s\", \"num_envs\": %d, \"horizon\": %d, \"grid\": %d, \"block\": %d, "
           "\"avg_us\": %.3f, \"bytes\": %.0f, \"gbs\": %.1f, \"frac_hbm\": %.4f}",
           first ? "" : ",\n", name, n, T, grid, block, us, bytes, bytes > 0 ? bytes / us * 1e-3 : 0.0,
           bytes > 0 ? bytes / us * 1e-3 / 8000.0 : 0.0);
    first = false;
  };
  {
    double *dq, *o;
    CK(hipMalloc(&dq, 64 * 8));
    CK(hipMalloc(&o, 1 << 20));
    std::vector<double> h(64);
    for (int i = 0; i < 64; ++i) h[i] = (i & 1) ? 0.97 : 0.01 * i;
    CK(hipMemcpy(dq, h.data(), 64 * 8, hipMemcpyHostToDevice));
    emit("chain_kernel<128>", 0, 256, 64, time_us(chain_kernel<128>, 256, 64, reps, (const double *)dq, o), 0.0);
    emit("chain_kernel<1024>", 0, 256, 64, time_us(chain_kernel<1024>, 256, 64, reps, (const double *)dq, o), 0.0);
    emit("chain_kernel<8192>", 0, 256, 64, time_us(chain_kernel<8192>, 256, 64, reps, (const double *)dq, o), 0.0);
  }
  for (int n : {4096, 16384, 65536}) {
    const int grid = n / 16;
    const double bytes = 25.0 * n * T;
    if (n == 4096) {
      emit("empty_kernel", n, grid, 256, time_us(empty_kernel, grid, 256, reps), 0.0);
      emit("ld1st1_kernel", n, grid, 256,
           time_us(ld1st1_kernel, grid, 256, reps, (const float *)B.in, B.out), 8.0 * grid * 256);
      emit("empty_kernel_1block", n, 1, 64, time_us(empty_kernel, 1, 64, reps), 0.0);
    }
    emit("scanbytes_kernel<16,8>", n, grid, 256,
         time_us(scanbytes_kernel<16, 8>, grid, 256, reps, (const float *)B.v, (const float *)B.vn,
                 (const double *)B.r, (const uint8_t *)B.term, (const uint8_t *)B.done, n, T, B.adv, B.vt),
         bytes);
    emit("scanbytes_kernel<4,8>", n, n / 4, 64,
         time_us(scanbytes_kernel<4, 8>, n / 4, 64, reps, (const float *)B.v, (const float *)B.vn,
                 (const double *)B.r, (const uint8_t *)B.term, (const uint8_t *)B.done, n, T, B.adv, B.vt),
         bytes);
  }
  printf("\n]\n");
  CK(hipDeviceSynchronize());
  return 0;
}
