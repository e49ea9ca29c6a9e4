// Diagnostic microbenchmark (not part of the library): what bounds a register scan of a DNA text that keys
// every position and keeps 1/8 of them (the slice pre-pass shape, k_slice_hist_spans REG).  Each variant adds
// one stage of that kernel; time per variant with HIP events over a 4 GiB buffer.
//   hipcc -O3 --offload-arch=gfx950 tools/scanbench.hip -o tools/scanbench && ./tools/scanbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int T = 1024, PER = 16, TILE = T * PER;

__device__ __forceinline__ uint32_t pack16(const uint4& v) {
  auto p8 = [&](uint32_t w) -> uint32_t {
    const uint32_t c = __builtin_amdgcn_perm(0x03020100u, 0x00010203u, w & 0x07070707u);
    return __builtin_amdgcn_udot4(c, 0x01041040u, 0u, false);
  };
  return (((p8(v.x) << 8) | p8(v.y)) << 16) | (p8(v.z) << 8) | p8(v.w);
}
__device__ __forceinline__ uint32_t win(uint32_t a, uint32_t b, int k) { return k ? __builtin_amdgcn_alignbit(a, b, 32 - 2 * k) : a; }

// MODE 0: loads only; 1: + pack; 2: + windows / test (count in a register); 3: + exec-masked u8 LDS adds
// (LDS = 128 KiB); 4: as 3 with LDS adds of all positions (no test); LDSW: words of LDS counters
template <int MODE, int PF, int LDSW>
__global__ __launch_bounds__(T, 1) void k_scan(const uint8_t* __restrict__ t, uint64_t span, uint32_t wb, uint32_t wn1,
                                               int dsh, uint32_t* __restrict__ out) {
  __shared__ uint32_t H[LDSW];
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < LDSW; i += T) H[i] = 0;
  __syncthreads();
  const uint64_t lo = (uint64_t)blockIdx.x * span, hi = lo + span;
  uint4 f0[PF], f1[PF];
  auto fetch = [&](uint64_t p, uint4& a, uint4& b) {
    const uint4* s = reinterpret_cast<const uint4*>(t + (p < hi ? p : lo));
    a = s[0];
    b = s[1];
  };
#pragma unroll
  for (int u = 0; u < PF; ++u) fetch(lo + (uint64_t)u * TILE + tid * PER, f0[u], f1[u]);
  uint32_t acc = 0;
  for (uint64_t base = lo; base < hi; base += PF * TILE) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const uint64_t p0 = base + (uint64_t)u * TILE + tid * PER;
      const uint4 a = f0[u], b = f1[u];
      if (MODE == 0) {
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x;
      } else {
        const uint32_t c0 = pack16(a), c1 = pack16(b);
        if (MODE == 1) {
          acc ^= c0 ^ c1;
        } else {
#pragma unroll
          for (int k = 0; k < PER; ++k) {
            const uint32_t w = win(c0, c1, k) - wb;
            if (MODE == 2) {
              acc += w <= wn1 ? 1u : 0u;
            } else if (MODE == 3) {
              if (w <= wn1) {
                const uint32_t bb = (w >> dsh) % (LDSW * 4);
                atomicAdd(&H[bb >> 2], 1u << (8 * (bb & 3)));
              }
            } else if (MODE == 4) {
              const uint32_t bb = (w >> dsh) % (LDSW * 4);
              atomicAdd(&H[bb >> 2], 1u << (8 * (bb & 3)));
            }
          }
          if (MODE == 5) {   // kept mask, then one add per kept position (max-over-lanes trips)
            uint32_t m = 0;
#pragma unroll
            for (int k = 0; k < PER; ++k) m = m + m + (win(c0, c1, k) - wb <= wn1 ? 1u : 0u);
            const uint32_t x0 = c0 >> 2, x1 = __builtin_amdgcn_alignbit(c0, c1, 2);
            while (m) {
              const uint32_t j = (uint32_t)__builtin_ctz(m);
              m &= m - 1;
              const uint32_t bb = ((__builtin_amdgcn_alignbit(x0, x1, 2 * j) - wb) >> dsh) % (LDSW * 4);
              atomicAdd(&H[bb >> 2], 1u << (8 * (bb & 3)));
            }
          }
          if (MODE == 6) {   // kept mask, then a fixed two-add pass per lane + a loop for the rest
            uint32_t m = 0;
#pragma unroll
            for (int k = 0; k < PER; ++k) m = m + m + (win(c0, c1, k) - wb <= wn1 ? 1u : 0u);
            const uint32_t x0 = c0 >> 2, x1 = __builtin_amdgcn_alignbit(c0, c1, 2);
            // two unconditional adds (a lane without a kept position adds 0 to its own dummy word)
            uint32_t a0, v0, a1, v1;
            {
              const uint32_t j = m ? (uint32_t)__builtin_ctz(m) : 0u;
              const uint32_t bb = ((__builtin_amdgcn_alignbit(x0, x1, 2 * j) - wb) >> dsh) % (LDSW * 4);
              a0 = m ? bb >> 2 : (LDSW - 64 + (tid & 63));
              v0 = m ? 1u << (8 * (bb & 3)) : 0u;
              m &= m - 1;
            }
            {
              const uint32_t j = m ? (uint32_t)__builtin_ctz(m) : 0u;
              const uint32_t bb = ((__builtin_amdgcn_alignbit(x0, x1, 2 * j) - wb) >> dsh) % (LDSW * 4);
              a1 = m ? bb >> 2 : (LDSW - 64 + (tid & 63));
              v1 = m ? 1u << (8 * (bb & 3)) : 0u;
              m &= m - 1;
            }
            atomicAdd(&H[a0], v0);
            atomicAdd(&H[a1], v1);
            while (m) {
              const uint32_t j = (uint32_t)__builtin_ctz(m);
              m &= m - 1;
              const uint32_t bb = ((__builtin_amdgcn_alignbit(x0, x1, 2 * j) - wb) >> dsh) % (LDSW * 4);
              atomicAdd(&H[bb >> 2], 1u << (8 * (bb & 3)));
            }
          }
        }
      }
      fetch(p0 + PF * TILE, f0[u], f1[u]);
    }
  }
  __syncthreads();
  if (MODE >= 3) acc += H[tid];
  out[(uint64_t)blockIdx.x * T + tid] = acc;
}

int main() {
  const uint64_t n = 4ull << 30;
  uint8_t* d;
  uint32_t* o;
  CK(hipMalloc(&d, n + 4096));
  CK(hipMalloc(&o, 4096ull * T * 4));
  std::vector<uint8_t> h(1 << 24);
  uint64_t x = 88172645463325252ull;
  for (auto& c : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; c = "ACGT"[x & 3]; }
  for (uint64_t off = 0; off < n; off += h.size()) CK(hipMemcpy(d + off, h.data(), h.size(), hipMemcpyHostToDevice));
  CK(hipMemset(d + n, 'A', 4096));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // window range [wb, wb + wn1]: the first eighth of the 32-bit window space; bins = the 15 bits below
  const uint32_t wb = 0x20000000u, wn1 = 0x1FFFFFFFu;
  auto run = [&](const char* name, auto kern, int grid) -> int {
    const uint64_t span = n / grid;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0));
      kern<<<grid, T>>>(d, span, wb, wn1, 14, o);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep == 2) printf("%-44s grid %5d  %7.3f ms  %6.2f TB/s of text\n", name, grid, ms, n / ms / 1e9);
    }
    return 0;
  };
  run("loads only PF4", k_scan<0, 4, 64>, 256);
  run("loads only PF4 (1024 WGs)", k_scan<0, 4, 64>, 1024);
  run("+ pack PF4", k_scan<1, 4, 64>, 256);
  run("+ windows/test PF4", k_scan<2, 4, 64>, 256);
  run("+ masked LDS adds (128 KiB) PF4", k_scan<3, 4, 32768>, 256);
  run("+ masked LDS adds (32 KiB, 4 WG/CU) PF4", k_scan<3, 4, 8192>, 1024);
  run("all-position LDS adds (128 KiB) PF4", k_scan<4, 4, 32768>, 256);
  run("+ windows/test PF8", k_scan<2, 8, 64>, 256);
  run("+ masked LDS adds (128 KiB) PF8", k_scan<3, 8, 32768>, 256);
  run("compacted adds (128 KiB) PF4", k_scan<5, 4, 32768>, 256);
  run("compacted adds (128 KiB) PF8", k_scan<5, 8, 32768>, 256);
  run("two fixed adds + loop (128 KiB) PF4", k_scan<6, 4, 32768>, 256);
  run("two fixed adds + loop (128 KiB) PF8", k_scan<6, 8, 32768>, 256);
  return 0;
}
