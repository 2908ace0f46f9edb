// Round 4 probe: (1) which XCD (HW_REG_XCC_ID) each workgroup of a launch of
// 8*P workgroups lands on; (2) the cost of a barrier among P workgroups that
// all run on one XCD (one shared L2: an atomic counter in L2, stores drained
// with s_waitcnt, this CU's L1 invalidated after the wait), with a data check
// that every participant sees the others' stores of the same round.  Every
// spin is bounded: a participant that waits too long sets err and leaves.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ int xcc_id() {
  // s_getreg_b32 hwreg(HW_REG_XCC_ID = 20, offset 0, size 4)
  return __builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11)) & 15;
}

__global__ void k_where(int* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = xcc_id();
}

constexpr long long kSpinLimit = 1ll << 22;

__device__ __forceinline__ bool xcd_barrier(unsigned* cnt, unsigned target, int* err) {
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0) in every wave: its stores have reached L2
  __syncthreads();
  bool ok = true;
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    long long it = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (++it > kSpinLimit) {
        *err = 1;
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  asm volatile("buffer_inv sc1" ::: "memory");   // this CU's L1, from every wave (v2/v3: one wave)
  return ok;
}

// the same with arrival flags: each participant stores its round number in
// its own word, participant 0 polls all of them with one wave (one word per
// lane) and then stores the round into the release word the others poll
__device__ __forceinline__ bool xcd_barrier2(unsigned* arrive, unsigned* release, int s, int P, unsigned round,
                                             int* err) {
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();
  bool ok = true;
  if (threadIdx.x == 0) __hip_atomic_store(arrive + 16 * s, round, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (s == 0 && threadIdx.x < 64) {
    long long it = 0;
    const int l = threadIdx.x;
    while (true) {
      const unsigned v = l < P ? __hip_atomic_load(arrive + 16 * l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : round;
      if (__all(v >= round)) break;
      if (++it > kSpinLimit) {
        if (l == 0) *err = 1;
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (l == 0) __hip_atomic_store(release, round, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if (threadIdx.x == 0) {
    long long it = 0;
    while (__hip_atomic_load(release, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < round) {
      if (++it > kSpinLimit) {
        *err = 1;
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  if (threadIdx.x < 64) asm volatile("buffer_inv sc1\n\ts_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  return ok;
}

// v4: v2 without the L1 invalidation; the payload is read with nt loads,
// which bypass L1 (served by the XCD's L2)
__device__ __forceinline__ bool xcd_barrier4(unsigned* arrive, unsigned* release, int s, int P, unsigned round,
                                             int* err) {
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();
  bool ok = true;
  if (threadIdx.x == 0) __hip_atomic_store(arrive + 16 * s, round, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (s == 0 && threadIdx.x < 64) {
    long long it = 0;
    const int l = threadIdx.x;
    while (true) {
      const unsigned v = l < P ? __hip_atomic_load(arrive + 16 * l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : round;
      if (__all(v >= round)) break;
      if (++it > kSpinLimit) {
        if (l == 0) *err = 1;
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (l == 0) __hip_atomic_store(release, round, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if (threadIdx.x == 0) {
    long long it = 0;
    while (__hip_atomic_load(release, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < round) {
      if (++it > kSpinLimit) {
        *err = 1;
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  return ok;
}

// v3: the flags through L2 only: plain stores (write through L1 into the
// XCD's L2), polls as group-scope loads (L1 bypassed)
__device__ __forceinline__ unsigned l2_load(const unsigned* p) {
  // a group-scope load (sc0): misses this CU's L1, served by the XCD's L2
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ bool xcd_barrier3(unsigned* arrive, unsigned* release, int s, int P, unsigned round,
                                             int* err) {
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();
  bool ok = true;
  if (threadIdx.x == 0) {
    *(volatile unsigned*)(arrive + 16 * s) = round;
    __builtin_amdgcn_s_waitcnt(0x0F70);
  }
  if (s == 0 && threadIdx.x < 64) {
    long long it = 0;
    const int l = threadIdx.x;
    while (true) {
      const unsigned v = l < P ? l2_load(arrive + 16 * l) : round;
      if (__all(v >= round)) break;
      if (++it > kSpinLimit) {
        if (l == 0) *err = 1;
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (l == 0) {
      *(volatile unsigned*)release = round;
      __builtin_amdgcn_s_waitcnt(0x0F70);
    }
  } else if (threadIdx.x == 0) {
    long long it = 0;
    while (l2_load(release) < round) {
      if (++it > kSpinLimit) {
        *err = 1;
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  if (threadIdx.x < 64) asm volatile("buffer_inv sc1\n\ts_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  return ok;
}

__global__ void __launch_bounds__(256) k_bar3(int P, int rounds, unsigned* ctr, double* data, long long* t,
                                              int* err, int* bad) {
  __shared__ int slot;
  if (xcc_id() != 0) return;
  if (threadIdx.x == 0) slot = (int)__hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int s = slot;
  if (s >= P) return;
  unsigned* arrive = ctr + 64;
  unsigned* release = ctr + 32;
  long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int r = 0; r < rounds; r++) {
    for (int q = threadIdx.x; q < 512; q += 256) data[(long long)s * 512 + q] = (double)(r * 100000 + s * 1000 + q);
    if (!xcd_barrier3(arrive, release, s, P, 2 * r + 1, err)) return;
    const int o = (s + 1) % P;
    for (int q = threadIdx.x; q < 512; q += 256)
      if (data[(long long)o * 512 + q] != (double)(r * 100000 + o * 1000 + q)) atomicAdd(bad, 1);
    if (!xcd_barrier3(arrive, release, s, P, 2 * r + 2, err)) return;
  }
  if (threadIdx.x == 0 && s == 0) t[0] = __builtin_amdgcn_s_memrealtime() - t0;
}

__global__ void __launch_bounds__(256) k_bar2(int P, int rounds, unsigned* ctr, double* data, long long* t,
                                              int* err, int* bad) {
  __shared__ int slot;
  if (xcc_id() != 0) return;
  if (threadIdx.x == 0) slot = (int)__hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int s = slot;
  if (s >= P) return;
  unsigned* arrive = ctr + 64;
  unsigned* release = ctr + 32;
  long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int r = 0; r < rounds; r++) {
    for (int q = threadIdx.x; q < 512; q += 256) data[(long long)s * 512 + q] = (double)(r * 100000 + s * 1000 + q);
    if (!xcd_barrier2(arrive, release, s, P, 2 * r + 1, err)) return;
    const int o = (s + 1) % P;
    for (int q = threadIdx.x; q < 512; q += 256)
      if (data[(long long)o * 512 + q] != (double)(r * 100000 + o * 1000 + q)) atomicAdd(bad, 1);
    if (!xcd_barrier2(arrive, release, s, P, 2 * r + 2, err)) return;
  }
  if (threadIdx.x == 0 && s == 0) t[0] = __builtin_amdgcn_s_memrealtime() - t0;
}

__global__ void __launch_bounds__(256) k_bar4(int P, int rounds, unsigned* ctr, double* data, long long* t,
                                              int* err, int* bad) {
  __shared__ int slot;
  if (xcc_id() != 0) return;
  if (threadIdx.x == 0) slot = (int)__hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int s = slot;
  if (s >= P) return;
  unsigned* arrive = ctr + 64;
  unsigned* release = ctr + 32;
  long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int r = 0; r < rounds; r++) {
    for (int q = threadIdx.x; q < 512; q += 256) data[(long long)s * 512 + q] = (double)(r * 100000 + s * 1000 + q);
    if (!xcd_barrier4(arrive, release, s, P, 2 * r + 1, err)) return;
    const int o = (s + 1) % P;
    for (int q = threadIdx.x; q < 512; q += 256)
      if (__builtin_nontemporal_load(&data[(long long)o * 512 + q]) != (double)(r * 100000 + o * 1000 + q)) atomicAdd(bad, 1);
    if (!xcd_barrier4(arrive, release, s, P, 2 * r + 2, err)) return;
  }
  if (threadIdx.x == 0 && s == 0) t[0] = __builtin_amdgcn_s_memrealtime() - t0;
}

__global__ void __launch_bounds__(256) k_bar(int P, int rounds, unsigned* ctr, double* data, long long* t,
                                             int* err, int* bad) {
  __shared__ int slot;
  if (xcc_id() != 0) return;
  if (threadIdx.x == 0) slot = (int)__hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int s = slot;
  if (s >= P) return;
  unsigned* cnt = ctr + 16;
  long long t0 = __builtin_amdgcn_s_memrealtime();
  // (the values are integers: exact whatever the compiler contracts)
  for (int r = 0; r < rounds; r++) {
    for (int q = threadIdx.x; q < 512; q += 256) data[(long long)s * 512 + q] = (double)(r * 100000 + s * 1000 + q);
    if (!xcd_barrier(cnt, (unsigned)(P * (r + 1)), err)) return;
    const int o = (s + 1) % P;
    for (int q = threadIdx.x; q < 512; q += 256)
      if (data[(long long)o * 512 + q] != (double)(r * 100000 + o * 1000 + q)) atomicAdd(bad, 1);
    if (!xcd_barrier(cnt + 16, (unsigned)(P * (r + 1)), err)) return;
  }
  if (threadIdx.x == 0 && s == 0) t[0] = __builtin_amdgcn_s_memrealtime() - t0;
}

int main() {
  int* d_where;
  (void)hipMalloc(&d_where, sizeof(int) * 4096);
  for (int n : {8, 64, 512}) {
    k_where<<<n, 64>>>(d_where);
    std::vector<int> h(n);
    (void)hipMemcpy(h.data(), d_where, sizeof(int) * n, hipMemcpyDeviceToHost);
    int cnt[16] = {}, rr = 0;
    for (int i = 0; i < n; i++) {
      cnt[h[i] & 15]++;
      rr += h[i] == i % 8;
    }
    std::printf("where n=%d: round-robin %d/%d, per xcc:", n, rr, n);
    for (int x = 0; x < 8; x++) std::printf(" %d", cnt[x]);
    std::printf("\n");
  }
  unsigned* ctr;
  double* data;
  long long* t;
  int *err, *bad;
  (void)hipMalloc(&ctr, 4096 * 4);
  (void)hipMalloc(&data, sizeof(double) * 512 * 64);
  (void)hipMalloc(&t, 8);
  (void)hipMalloc(&err, 4);
  (void)hipMalloc(&bad, 4);
  for (int v = 1; v <= 4; v++)
  for (int P : {8, 32, 64}) {
    const int rounds = 200;
    (void)hipMemset(ctr, 0, 4096);
    (void)hipMemset(err, 0, 4);
    (void)hipMemset(bad, 0, 4);
    (void)hipMemset(t, 0, 8);
    (void)hipMemset(ctr, 0, 4096 * 4);
    if (v == 1)
      k_bar<<<8 * P, 256>>>(P, rounds, ctr, data, t, err, bad);
    else if (v == 2)
      k_bar2<<<8 * P, 256>>>(P, rounds, ctr, data, t, err, bad);
    else if (v == 3)
      k_bar3<<<8 * P, 256>>>(P, rounds, ctr, data, t, err, bad);
    else
      k_bar4<<<8 * P, 256>>>(P, rounds, ctr, data, t, err, bad);
    (void)hipDeviceSynchronize();
    long long ht;
    int he, hb;
    (void)hipMemcpy(&ht, t, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    std::printf("barrier v%d P=%d: %.3f us per barrier (2 per round, %d rounds), err %d, stale reads %d\n", v, P,
                ht * 0.01 / (2.0 * rounds), rounds, he, hb);
  }
  return 0;
}
