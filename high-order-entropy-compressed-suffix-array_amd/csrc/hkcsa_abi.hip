// hkcsa_abi.hip — extern "C" boundary of libhkcsa.so (declared in include/hkcsa.h).
// Each entry point catches every C++ exception and maps it to a negative error code plus a
// thread-local message; nothing ever throws across the ABI.

#include <algorithm>
#include <cstring>
#include <initializer_list>
#include <memory>
#include <vector>
#include <new>
#include <string>

#include "../../include/hkcsa.h"
#include "hk_index.hpp"

struct hkcsa_queries {
  uint64_t P = 0, bytes = 0;
  hk::DevBuf pats, offs, lr, cnt, occ_offs, pos, flag;
  uint64_t total = 0;
  bool have_lr = false, have_pos = false;
  void release() {
    for (hk::DevBuf* b : {&pats, &offs, &lr, &cnt, &occ_offs, &pos, &flag}) b->release();
    have_lr = have_pos = false;
  }
  // the per-handle batch workspace keeps what an ordinary call needs; a buffer a large call grew past
  // kKeep is freed when that call ends, so one big locate does not pin HBM for the handle's lifetime
  static constexpr size_t kKeep = 64ull << 20;
  void trim() {
    for (hk::DevBuf* b : {&pats, &offs, &lr, &cnt, &occ_offs, &pos})
      if (b->bytes > kKeep) b->release();
  }
};

struct hkcsa_index {
  hk::Index ix;
  hkcsa_queries qws;                   // device workspace of the host-boundary batch calls, kept across calls
  hipStream_t copy_stream = nullptr;   // their pattern uploads (created on first use)
  hipEvent_t copy_ev = nullptr;
};

namespace hk {
static thread_local std::string g_err;
void set_error(const std::string& m) { g_err = m; }
}  // namespace hk

namespace {

template <typename F>
int guarded(F&& f) {
  try {
    f();
    return HKCSA_OK;
  } catch (const hk::HipError& e) {
    hk::set_error(std::string("HIP error ") + hipGetErrorString(e.code) + " in " + e.where);
    (void)hipGetLastError();
    return HKCSA_E_HIP;
  } catch (const hk::ApiError& e) {
    hk::set_error(e.msg);
    return e.code;
  } catch (const std::bad_alloc&) {
    hk::set_error("host allocation failed");
    return HKCSA_E_NOMEM;
  } catch (const std::exception& e) {
    hk::set_error(e.what());
    return HKCSA_E_INVALID;
  }
}

void need(bool c, int code, const char* msg) {
  if (!c) throw hk::ApiError{code, msg};
}

void activate(const hkcsa_index* h) {
  need(h != nullptr, HKCSA_E_INVALID, "null index handle");
  HK_HIP(hipSetDevice(h->ix.device));
}

void init_index(hk::Index& ix, const hkcsa_opts* o, uint64_t n) {
  int dev = (o && o->device >= 0) ? o->device : -1;
  if (dev < 0) HK_HIP(hipGetDevice(&dev));
  int cnt = 0;
  HK_HIP(hipGetDeviceCount(&cnt));
  need(dev < cnt, HKCSA_E_INVALID, "device ordinal out of range");
  HK_HIP(hipSetDevice(dev));
  ix.device = dev;
  ix.flags = o ? o->flags : 0u;
  HK_HIP(hipStreamCreateWithFlags(&ix.stream, hipStreamNonBlocking));
  ix.timer.stream = ix.stream;
  ix.n = n;
  ix.text.ensure(n + 64);
  HK_HIP(hipMemsetAsync(ix.text.p, 0, n + 64, ix.stream));
}

}  // namespace

extern "C" {

int hkcsa_abi_version(void) { return HKCSA_ABI_VERSION; }

const char* hkcsa_last_error(void) { return hk::g_err.c_str(); }

int hkcsa_device_count(int* n) {
  return guarded([&] {
    need(n != nullptr, HKCSA_E_INVALID, "null output");
    HK_HIP(hipGetDeviceCount(n));
  });
}

int hkcsa_create(const uint8_t* text, uint64_t n, const hkcsa_opts* o, hkcsa_index** out) {
  return guarded([&] {
    need(out != nullptr, HKCSA_E_INVALID, "null output handle");
    need(n == 0 || text != nullptr, HKCSA_E_INVALID, "null text");
    need(n > 0, HKCSA_E_INVALID, "text must hold at least the sentinel");
    auto* h = new hkcsa_index();
    try {
      init_index(h->ix, o, n);
      HK_HIP(hipMemcpyAsync(h->ix.text.p, text, n, hipMemcpyHostToDevice, h->ix.stream));
      HK_HIP(hipStreamSynchronize(h->ix.stream));
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int hkcsa_create_parts(const uint8_t* const* parts, const uint64_t* lens, int nparts, const hkcsa_opts* o,
                       hkcsa_index** out) {
  return guarded([&] {
    need(out != nullptr, HKCSA_E_INVALID, "null output handle");
    need(nparts >= 1 && parts != nullptr && lens != nullptr, HKCSA_E_INVALID, "no parts");
    uint64_t n = 0;
    for (int i = 0; i < nparts; ++i) {
      need(lens[i] == 0 || parts[i] != nullptr, HKCSA_E_INVALID, "null part");
      n += lens[i];
    }
    need(n > 0, HKCSA_E_INVALID, "text must hold at least the sentinel");
    auto* h = new hkcsa_index();
    try {
      init_index(h->ix, o, n);
      uint64_t at = 0;
      for (int i = 0; i < nparts; ++i) {
        if (lens[i])
          HK_HIP(hipMemcpyAsync(h->ix.text.as<uint8_t>() + at, parts[i], lens[i], hipMemcpyHostToDevice,
                                h->ix.stream));
        at += lens[i];
      }
      HK_HIP(hipStreamSynchronize(h->ix.stream));
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int hkcsa_create_synthetic(uint64_t n, const uint8_t* alphabet, int sigma, uint64_t seed,
                           uint8_t terminator, const hkcsa_opts* o, hkcsa_index** out) {
  return guarded([&] {
    need(out != nullptr, HKCSA_E_INVALID, "null output handle");
    need(n > 0, HKCSA_E_INVALID, "n must be > 0");
    need(alphabet != nullptr && sigma >= 1 && sigma <= 256, HKCSA_E_INVALID, "bad alphabet");
    auto* h = new hkcsa_index();
    try {
      init_index(h->ix, o, n);
      hk::synth_text(h->ix.text.as<uint8_t>(), n, alphabet, sigma, seed, terminator, h->ix.stream);
      HK_HIP(hipStreamSynchronize(h->ix.stream));
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int hkcsa_build_sa(hkcsa_index* h) {
  return guarded([&] {
    activate(h);
    need(h->ix.have_text, HKCSA_E_STATE, "text released by hkcsa_compact");
    h->ix.have_bwt = h->ix.have_wt = false;
    hk::build_sa(h->ix);
  });
}
int hkcsa_build_bwt(hkcsa_index* h) {
  return guarded([&] {
    activate(h);
    need(h->ix.have_text, HKCSA_E_STATE, "text released by hkcsa_compact");
    h->ix.have_wt = false;
    hk::build_bwt(h->ix);
  });
}
int hkcsa_build_wt(hkcsa_index* h) {
  return guarded([&] {
    activate(h);
    need(!h->ix.sharded, HKCSA_E_STATE, "sharded index holds only a slice: hkcsa_shard_replicate first");
    if (h->ix.bwt_in_wt) return;   // compacted: the WT is the only copy of the BWT
    hk::build_wt(h->ix);
  });
}
int hkcsa_build_all(hkcsa_index* h) {
  return guarded([&] {
    activate(h);
    need(h->ix.have_text, HKCSA_E_STATE, "text released by hkcsa_compact");
    hk::build_sa(h->ix);
    hk::build_bwt(h->ix);
    hk::build_wt(h->ix);
  });
}
int hkcsa_release_workspace(hkcsa_index* h) {
  return guarded([&] {
    activate(h);
    HK_HIP(hipStreamSynchronize(h->ix.stream));
    if (h->copy_stream) HK_HIP(hipStreamSynchronize(h->copy_stream));
    hk::release_workspace(h->ix);
    h->qws.release();   // the host-boundary batch calls' workspace too
  });
}
int hkcsa_build_samples(hkcsa_index* h, uint32_t rate) {
  return guarded([&] {
    activate(h);
    need(rate >= 1, HKCSA_E_INVALID, "sample rate must be >= 1");
    need(h->ix.have_text, HKCSA_E_STATE, "text released by hkcsa_compact");
    need(h->ix.have_sa && !h->ix.sharded, HKCSA_E_STATE, "suffix array not built");
    if (!h->ix.have_bwt) hk::build_bwt(h->ix);
    hk::build_samples(h->ix, rate);
  });
}

int hkcsa_entropy(hkcsa_index* h, int k, double* out) {
  return guarded([&] {
    activate(h);
    need(out != nullptr, HKCSA_E_INVALID, "null output");
    need(h->ix.have_text || k <= 0, HKCSA_E_STATE, "text released by hkcsa_compact");
    need(!h->ix.sharded || k <= 0, HKCSA_E_STATE, "sharded index holds only a slice");
    *out = hk::entropy_k(h->ix, k);
  });
}

int hkcsa_compact(hkcsa_index* h) {
  return guarded([&] {
    activate(h);
    need(h->ix.have_samples, HKCSA_E_STATE, "build the SA samples first");
    hk::compact(h->ix);
  });
}

int hkcsa_space(hkcsa_index* h, uint64_t out[8]) {
  return guarded([&] {
    activate(h);
    need(out != nullptr, HKCSA_E_INVALID, "null output");
    const hk::Index& ix = h->ix;
    const uint64_t nl = ix.n / hk::kLineBits + 1;
    out[0] = ix.have_text ? ix.n : 0;
    out[1] = ix.have_sa ? ix.n * (ix.sa_pos64 ? 8 : 4) : 0;
    out[2] = (ix.have_bwt && !ix.bwt_in_wt) ? ix.n : 0;
    out[3] = ix.have_wt ? (uint64_t)ix.wt_levels * nl * 64 : 0;
    out[4] = ix.have_samples ? nl * 64 : 0;
    out[5] = ix.have_samples ? (ix.smp_count * 2 + ix.smp_fixn) * (ix.smp_w64 ? 8 : 4) : 0;
    out[6] = ix.smp_rate;
    out[7] = ix.have_samples ? 1 : 0;
  });
}

int hkcsa_synchronize(hkcsa_index* h) {
  return guarded([&] {
    activate(h);
    HK_HIP(hipStreamSynchronize(h->ix.stream));
  });
}
void hkcsa_free(hkcsa_index* h) {
  if (!h) return;
  (void)hipSetDevice(h->ix.device);
  (void)hipStreamSynchronize(h->ix.stream);
  if (h->ix.aux_stream) (void)hipStreamSynchronize(h->ix.aux_stream);
  hipStream_t s = h->ix.stream, a = h->ix.aux_stream, cs = h->copy_stream;
  hipEvent_t ge = h->ix.geom_ev, ce = h->copy_ev;
  if (cs) (void)hipStreamSynchronize(cs);
  delete h;
  if (ge) (void)hipEventDestroy(ge);
  if (ce) (void)hipEventDestroy(ce);
  if (cs) (void)hipStreamDestroy(cs);
  if (s) (void)hipStreamDestroy(s);
  if (a) (void)hipStreamDestroy(a);
}

int hkcsa_bwt_gather(const uint8_t* text, uint64_t n, const uint64_t* sa, uint8_t* out) {
  return guarded([&] {
    need(n == 0 || (text && sa && out), HKCSA_E_INVALID, "null argument");
    if (!n) return;
    for (uint64_t i = 0; i < n; ++i) need(sa[i] < n, HKCSA_E_RANGE, "suffix array entry out of range");
    hk::Index ix;
    init_index(ix, nullptr, n);
    hipStream_t s = ix.stream;
    try {
      HK_HIP(hipMemcpyAsync(ix.text.p, text, n, hipMemcpyHostToDevice, s));
      hk::DevBuf dsa;
      dsa.ensure(n * 8);
      HK_HIP(hipMemcpyAsync(dsa.p, sa, n * 8, hipMemcpyHostToDevice, s));
      hk::bwt_gather64(ix, dsa.as<uint64_t>());
      HK_HIP(hipMemcpyAsync(out, ix.bwt.p, n, hipMemcpyDeviceToHost, s));
      HK_HIP(hipStreamSynchronize(s));
    } catch (...) {
      (void)hipStreamSynchronize(s);
      (void)hipStreamDestroy(s);
      throw;
    }
    (void)hipStreamDestroy(s);
  });
}

int hkcsa_use_text_as_bwt(hkcsa_index* h) {
  return guarded([&] {
    activate(h);
    need(h->ix.have_text, HKCSA_E_STATE, "text released by hkcsa_compact");
    h->ix.bwt.ensure(h->ix.n + 64);
    HK_HIP(hipMemcpyAsync(h->ix.bwt.p, h->ix.text.p, h->ix.n, hipMemcpyDeviceToDevice, h->ix.stream));
    HK_HIP(hipStreamSynchronize(h->ix.stream));
    h->ix.have_bwt = true;
    h->ix.have_wt = false;
  });
}

int hkcsa_get_n(const hkcsa_index* h, uint64_t* n) {
  return guarded([&] {
    need(h && n, HKCSA_E_INVALID, "null argument");
    *n = h->ix.n;
  });
}

int hkcsa_get_sa(hkcsa_index* h, uint64_t lo, uint64_t hi, uint64_t* out) {
  return guarded([&] {
    activate(h);
    need((h->ix.have_sa || h->ix.have_samples) && !h->ix.sharded, HKCSA_E_STATE, "suffix array not built");
    need(lo <= hi && hi <= h->ix.n, HKCSA_E_RANGE, "SA range out of bounds");
    need(hi == lo || out, HKCSA_E_INVALID, "null output");
    const uint64_t c = hi - lo;
    if (!c) return;
    if (!h->ix.have_sa) {   // compressed mode: LF walks to the samples
      hk::DevBuf tmp;
      tmp.ensure(c * 8);
      hk::sampled_sa_range(h->ix, lo, c, tmp.as<uint64_t>());
      HK_HIP(hipMemcpyAsync(out, tmp.p, c * 8, hipMemcpyDeviceToHost, h->ix.stream));
      HK_HIP(hipStreamSynchronize(h->ix.stream));
      return;
    }
    if (h->ix.sa_pos64) {   // replicated sharded SA of a text with n >= 2^32
      HK_HIP(hipMemcpyAsync(out, h->ix.sa.as<uint64_t>() + lo, c * 8, hipMemcpyDeviceToHost, h->ix.stream));
      HK_HIP(hipStreamSynchronize(h->ix.stream));
      return;
    }
    hk::sa_to_host_u64(h->ix, lo, c, out);
  });
}

int hkcsa_get_bwt(hkcsa_index* h, uint64_t lo, uint64_t hi, uint8_t* out) {
  return guarded([&] {
    activate(h);
    need(h->ix.have_bwt && !h->ix.sharded, HKCSA_E_STATE, "BWT not built (a sharded index holds only a slice)");
    need(lo <= hi && hi <= h->ix.n, HKCSA_E_RANGE, "BWT range out of bounds");
    if (hi == lo) return;
    need(out != nullptr, HKCSA_E_INVALID, "null output");
    if (h->ix.bwt_in_wt) {
      hk::DevBuf tmp;
      tmp.ensure(hi - lo);
      hk::wt_bwt_range(h->ix, lo, hi - lo, tmp.as<uint8_t>());
      HK_HIP(hipMemcpyAsync(out, tmp.p, hi - lo, hipMemcpyDeviceToHost, h->ix.stream));
      HK_HIP(hipStreamSynchronize(h->ix.stream));
      return;
    }
    HK_HIP(hipMemcpyAsync(out, h->ix.bwt.as<uint8_t>() + lo, hi - lo, hipMemcpyDeviceToHost, h->ix.stream));
    HK_HIP(hipStreamSynchronize(h->ix.stream));
  });
}

int hkcsa_get_text(hkcsa_index* h, uint64_t lo, uint64_t hi, uint8_t* out) {
  return guarded([&] {
    activate(h);
    need(lo <= hi && hi <= h->ix.n, HKCSA_E_RANGE, "text range out of bounds");
    if (hi == lo) return;
    need(out != nullptr, HKCSA_E_INVALID, "null output");
    if (!h->ix.have_text) {   // compressed mode: LF walks from the ISA samples
      hk::DevBuf tmp;
      tmp.ensure(hi - lo);
      hk::sampled_extract(h->ix, lo, hi, tmp.as<uint8_t>());
      HK_HIP(hipMemcpyAsync(out, tmp.p, hi - lo, hipMemcpyDeviceToHost, h->ix.stream));
      HK_HIP(hipStreamSynchronize(h->ix.stream));
      return;
    }
    HK_HIP(hipMemcpyAsync(out, h->ix.text.as<uint8_t>() + lo, hi - lo, hipMemcpyDeviceToHost, h->ix.stream));
    HK_HIP(hipStreamSynchronize(h->ix.stream));
  });
}

int hkcsa_extract(hkcsa_index* h, uint64_t i, uint64_t j, uint8_t* out) { return hkcsa_get_text(h, i, j, out); }

int hkcsa_get_C(hkcsa_index* h, uint64_t C[257]) {
  return guarded([&] {
    activate(h);
    need(C != nullptr, HKCSA_E_INVALID, "null output");
    hk::compute_alphabet(h->ix);
    memcpy(C, h->ix.Cbyte, 257 * 8);
  });
}

int hkcsa_get_alphabet(hkcsa_index* h, uint8_t syms[256], int* sigma) {
  return guarded([&] {
    activate(h);
    need(syms && sigma, HKCSA_E_INVALID, "null output");
    hk::compute_alphabet(h->ix);
    memcpy(syms, h->ix.syms, 256);
    *sigma = h->ix.sigma;
  });
}

int hkcsa_wt_levels(hkcsa_index* h, int* levels) {
  return guarded([&] {
    activate(h);
    need(levels != nullptr, HKCSA_E_INVALID, "null output");
    need(h->ix.have_wt, HKCSA_E_STATE, "wavelet tree not built");
    *levels = h->ix.wt_levels;
  });
}

int hkcsa_wt_level(hkcsa_index* h, int depth, uint64_t* nbits, uint64_t* words_out) {
  return guarded([&] {
    activate(h);
    need(h->ix.have_wt, HKCSA_E_STATE, "wavelet tree not built");
    need(depth >= 0 && depth < h->ix.wt_levels, HKCSA_E_RANGE, "level out of range");
    if (nbits) *nbits = h->ix.n;
    if (!words_out) return;
    const uint64_t nw = hk::ceil_div(h->ix.n, 64);
    hk::DevBuf tmp;
    tmp.ensure(nw * 8 + 8);
    hk::wt_level_words(h->ix, depth, tmp.as<uint64_t>());
    HK_HIP(hipMemcpyAsync(words_out, tmp.p, nw * 8, hipMemcpyDeviceToHost, h->ix.stream));
    HK_HIP(hipStreamSynchronize(h->ix.stream));
  });
}

int hkcsa_wt_golomb(hkcsa_index* h, int depth, uint64_t nbits, uint32_t m_override, uint32_t* m_out,
                    uint64_t* ones_out, uint64_t* code_bits, uint64_t* words_out, uint64_t cap_words) {
  return guarded([&] {
    activate(h);
    need(h->ix.have_wt, HKCSA_E_STATE, "wavelet tree not built");
    need(depth >= 0 && depth < h->ix.wt_levels, HKCSA_E_RANGE, "level out of range");
    need(nbits <= h->ix.n, HKCSA_E_RANGE, "prefix longer than the level");
    need(m_override < 64, HKCSA_E_INVALID, "m must be below 64");
    const hk::GolombResult r = hk::wt_golomb(h->ix, depth, nbits, m_override, words_out != nullptr);
    if (m_out) *m_out = r.m;
    if (ones_out) *ones_out = r.ones;
    if (code_bits) *code_bits = r.bits;
    if (!words_out) return;
    const uint64_t nw = hk::ceil_div(r.bits, 64);
    need(cap_words >= nw, HKCSA_E_RANGE, "output buffer too small for the code");
    if (nw) {
      HK_HIP(hipMemcpyAsync(words_out, h->ix.gr_out.p, nw * 8, hipMemcpyDeviceToHost, h->ix.stream));
      HK_HIP(hipStreamSynchronize(h->ix.stream));
    }
  });
}

int hkcsa_rank(hkcsa_index* h, const uint8_t* c, const uint64_t* i, uint64_t count, uint64_t* out) {
  return guarded([&] {
    activate(h);
    need(h->ix.have_wt && !h->ix.sharded, HKCSA_E_STATE, "wavelet tree not built");
    if (!count) return;
    need(c && i && out, HKCSA_E_INVALID, "null argument");
    hk::DevBuf dc, di, dout;
    dc.ensure(count);
    di.ensure(count * 8);
    dout.ensure(count * 8);
    hipStream_t s = h->ix.stream;
    HK_HIP(hipMemcpyAsync(dc.p, c, count, hipMemcpyHostToDevice, s));
    HK_HIP(hipMemcpyAsync(di.p, i, count * 8, hipMemcpyHostToDevice, s));
    hk::query_rank(h->ix, dc.as<uint8_t>(), di.as<uint64_t>(), count, dout.as<uint64_t>());
    HK_HIP(hipMemcpyAsync(out, dout.p, count * 8, hipMemcpyDeviceToHost, s));
    HK_HIP(hipStreamSynchronize(s));
  });
}

// ------------------------------------------------------------ query sets
int hkcsa_queries_upload(hkcsa_index* h, const uint8_t* pats, const uint64_t* offs, uint64_t P,
                         hkcsa_queries** out) {
  return guarded([&] {
    activate(h);
    need(out != nullptr, HKCSA_E_INVALID, "null output");
    need(offs != nullptr, HKCSA_E_INVALID, "null offsets");
    need(offs[0] == 0, HKCSA_E_INVALID, "offs[0] must be 0");
    for (uint64_t p = 0; p < P; ++p) need(offs[p + 1] >= offs[p], HKCSA_E_INVALID, "offsets not monotone");
    const uint64_t bytes = offs[P];
    need(bytes == 0 || pats != nullptr, HKCSA_E_INVALID, "null patterns");
    auto* q = new hkcsa_queries();
    try {
      hipStream_t s = h->ix.stream;
      q->P = P;
      q->bytes = bytes;
      q->flag.ensure(16);
      q->pats.ensure(bytes + 16);
      q->offs.ensure((P + 1) * 8);
      if (bytes) HK_HIP(hipMemcpyAsync(q->pats.p, pats, bytes, hipMemcpyHostToDevice, s));
      HK_HIP(hipMemcpyAsync(q->offs.p, offs, (P + 1) * 8, hipMemcpyHostToDevice, s));
      q->lr.ensure(P * 16 + 16);
      q->cnt.ensure(P * 8 + 16);
      q->occ_offs.ensure((P + 1) * 8 + 16);
      HK_HIP(hipStreamSynchronize(s));
    } catch (...) {
      delete q;
      throw;
    }
    *out = q;
  });
}

int hkcsa_queries_count(hkcsa_index* h, hkcsa_queries* q) {
  return guarded([&] {
    activate(h);
    need(q != nullptr, HKCSA_E_INVALID, "null query set");
    need(!h->ix.sharded, HKCSA_E_STATE, "sharded index holds only a slice");
    hk::query_count(h->ix, q->pats.as<uint8_t>(), q->offs.as<uint64_t>(), q->P, q->lr.as<int64_t>(),
                    q->cnt.as<uint64_t>(), q->bytes, q->flag.as<uint32_t>());
    q->have_lr = true;
    q->have_pos = false;
  });
}

int hkcsa_queries_locate(hkcsa_index* h, hkcsa_queries* q, uint64_t* total) {
  return guarded([&] {
    activate(h);
    need(q != nullptr, HKCSA_E_INVALID, "null query set");
    need(!h->ix.sharded, HKCSA_E_STATE, "sharded index holds only a slice");
    hipStream_t s = h->ix.stream;
    hk::query_count(h->ix, q->pats.as<uint8_t>(), q->offs.as<uint64_t>(), q->P, q->lr.as<int64_t>(),
                    q->cnt.as<uint64_t>(), q->bytes, q->flag.as<uint32_t>());
    hk::scan_exclusive_u64(h->ix.sw, q->cnt.as<uint64_t>(), q->occ_offs.as<uint64_t>(), q->P, true, s);
    uint64_t tot = 0;
    HK_HIP(hipMemcpyAsync(&tot, q->occ_offs.as<uint64_t>() + q->P, 8, hipMemcpyDeviceToHost, s));
    HK_HIP(hipStreamSynchronize(s));
    q->pos.ensure(tot * 8 + 16);
    hk::query_locate_gather(h->ix, q->lr.as<int64_t>(), q->occ_offs.as<uint64_t>(), q->P, q->pos.as<uint64_t>());
    q->total = tot;
    q->have_lr = q->have_pos = true;
    if (total) *total = tot;
  });
}

int hkcsa_queries_download(hkcsa_index* h, hkcsa_queries* q, int64_t* lr_out, uint64_t* occ_offs,
                           uint64_t* pos_out, uint64_t cap) {
  return guarded([&] {
    activate(h);
    need(q != nullptr, HKCSA_E_INVALID, "null query set");
    need(q->have_lr, HKCSA_E_STATE, "queries not run");
    hipStream_t s = h->ix.stream;
    if (lr_out && q->P) HK_HIP(hipMemcpyAsync(lr_out, q->lr.p, q->P * 16, hipMemcpyDeviceToHost, s));
    if (occ_offs || pos_out) need(q->have_pos, HKCSA_E_STATE, "locate not run");
    if (occ_offs) HK_HIP(hipMemcpyAsync(occ_offs, q->occ_offs.p, (q->P + 1) * 8, hipMemcpyDeviceToHost, s));
    if (pos_out && q->total) {
      need(cap >= q->total, HKCSA_E_RANGE, "position buffer too small");
      HK_HIP(hipMemcpyAsync(pos_out, q->pos.p, q->total * 8, hipMemcpyDeviceToHost, s));
    }
    HK_HIP(hipStreamSynchronize(s));
  });
}

void hkcsa_queries_free(hkcsa_queries* q) { delete q; }

}  // extern "C"

namespace {
// Host-boundary batch calls.  The caller's buffers are pageable; HIP's own pageable copies run at PCIe rate on
// MI355X hosts (24 MB up in 0.43 ms, the same as from pinned memory, and 0.64 ms less than the round-5
// threaded pinned staging), so the calls copy straight from and into them.  The upload goes in chunks of
// kCountChunk patterns on the handle's copy stream, and the count of a chunk is queued on the handle's stream
// behind its chunk's copies: counting chunk c overlaps uploading chunk c + 1.  The offsets are checked by
// the count kernel itself (a pattern whose end precedes its start or passes offs[P] is not read and raises
// the query set's flag, read back before any result leaves the device), not by a host pass over them.
constexpr uint64_t kCountChunk = 1ull << 18;

hkcsa_queries& batch_count(hkcsa_index* h, const uint8_t* pats, const uint64_t* offs, uint64_t P) {
  need(offs != nullptr, HKCSA_E_INVALID, "null offsets");
  need(offs[0] == 0, HKCSA_E_INVALID, "offs[0] must be 0");
  const uint64_t bytes = offs[P];
  need(bytes == 0 || pats != nullptr, HKCSA_E_INVALID, "null patterns");
  hkcsa_queries& q = h->qws;
  q.P = P;
  q.bytes = bytes;
  q.total = 0;
  q.have_lr = q.have_pos = false;
  q.pats.ensure(bytes + 16);
  q.offs.ensure((P + 1) * 8);
  q.lr.ensure(P * 16 + 16);
  q.cnt.ensure(P * 8 + 16);
  q.occ_offs.ensure((P + 1) * 8 + 16);
  q.flag.ensure(16);
  hipStream_t s = h->ix.stream;
  if (!h->copy_stream) HK_HIP(hipStreamCreateWithFlags(&h->copy_stream, hipStreamNonBlocking));
  if (!h->copy_ev) HK_HIP(hipEventCreateWithFlags(&h->copy_ev, hipEventDisableTiming));
  hipStream_t cs = h->copy_stream;
  HK_HIP(hipMemsetAsync(q.flag.p, 0, 4, s));
  // the uploads start behind everything already queued on the handle (earlier kernels read these buffers)
  HK_HIP(hipEventRecord(h->copy_ev, s));
  HK_HIP(hipStreamWaitEvent(cs, h->copy_ev, 0));
  uint8_t* const dp = q.pats.as<uint8_t>();
  uint64_t* const dofs = q.offs.as<uint64_t>();
  try {
    for (uint64_t p0 = 0; p0 < P || p0 == 0; p0 += kCountChunk) {
      const uint64_t p1 = std::min(P, p0 + kCountChunk);
      // this chunk's pattern bytes (clamped: offsets out of order only lose bytes the kernel will not read)
      const uint64_t b0 = std::min(offs[p0], bytes), b1 = std::min(std::max(offs[p1], b0), bytes);
      if (b1 > b0) HK_HIP(hipMemcpyAsync(dp + b0, pats + b0, b1 - b0, hipMemcpyHostToDevice, cs));
      HK_HIP(hipMemcpyAsync(dofs + p0, offs + p0, (p1 - p0 + 1) * 8, hipMemcpyHostToDevice, cs));
      HK_HIP(hipEventRecord(h->copy_ev, cs));
      HK_HIP(hipStreamWaitEvent(s, h->copy_ev, 0));
      hk::query_count(h->ix, dp, dofs + p0, p1 - p0, q.lr.as<int64_t>() + 2 * p0, q.cnt.as<uint64_t>() + p0, bytes,
                      q.flag.as<uint32_t>());
      if (p1 >= P) break;
    }
  } catch (...) {
    // copies from the caller's buffers may still be queued: drain both streams before the error returns,
    // so the caller may free them (their own errors are superseded by this one)
    (void)hipStreamSynchronize(cs);
    (void)hipStreamSynchronize(s);
    throw;
  }
  return q;
}

// the count kernels' offsets flag, landed in the pinned read-back slot rb[4] (the caller synchronizes)
void flag_readback(hkcsa_index* h, hkcsa_queries& q) {
  uint64_t* const rb = h->ix.rb();
  rb[4] = 0;
  HK_HIP(hipMemcpyAsync(&rb[4], q.flag.p, 4, hipMemcpyDeviceToHost, h->ix.stream));
}
void flag_check(hkcsa_index* h) {
  need(h->ix.rb()[4] == 0, HKCSA_E_INVALID, "offsets not monotone (or past offs[P])");
}
}  // namespace

extern "C" {

int hkcsa_count_batch(hkcsa_index* h, const uint8_t* pats, const uint64_t* offs, uint64_t P, int64_t* lr_out) {
  return guarded([&] {
    activate(h);
    need(lr_out != nullptr || P == 0, HKCSA_E_INVALID, "null output");
    need(!h->ix.sharded, HKCSA_E_STATE, "sharded index holds only a slice");
    hkcsa_queries& q = batch_count(h, pats, offs, P);
    hipStream_t s = h->ix.stream;
    flag_readback(h, q);
    HK_HIP(hipStreamSynchronize(s));
    flag_check(h);
    if (P) HK_HIP(hipMemcpyAsync(lr_out, q.lr.p, P * 16, hipMemcpyDeviceToHost, s));
    HK_HIP(hipStreamSynchronize(s));
    q.trim();
  });
}

// Sizes first (count + scan, no gather); the SA gather runs only when pos_out can hold every
// position, so a caller with a large enough buffer finishes in one call and a short one gets the
// CSR offsets with HKCSA_E_RANGE (nothing gathered) and calls again.
int hkcsa_locate_batch(hkcsa_index* h, const uint8_t* pats, const uint64_t* offs, uint64_t P,
                       uint64_t* occ_offs, uint64_t* pos_out, uint64_t cap) {
  return guarded([&] {
    activate(h);
    need(occ_offs != nullptr, HKCSA_E_INVALID, "null occ_offs");
    need(!h->ix.sharded, HKCSA_E_STATE, "sharded index holds only a slice");
    hkcsa_queries& q = batch_count(h, pats, offs, P);
    hipStream_t s = h->ix.stream;
    hk::scan_exclusive_u64(h->ix.sw, q.cnt.as<uint64_t>(), q.occ_offs.as<uint64_t>(), q.P, true, s);
    uint64_t* const rb = h->ix.rb();   // pinned: the total and the offsets flag in one round trip
    HK_HIP(hipMemcpyAsync(&rb[3], q.occ_offs.as<uint64_t>() + P, 8, hipMemcpyDeviceToHost, s));
    flag_readback(h, q);
    HK_HIP(hipStreamSynchronize(s));
    flag_check(h);
    const uint64_t tot = rb[3];
    if (pos_out && cap >= tot && tot) {
      q.pos.ensure(tot * 8 + 16);
      hk::query_locate_gather(h->ix, q.lr.as<int64_t>(), q.occ_offs.as<uint64_t>(), q.P, q.pos.as<uint64_t>());
    }
    HK_HIP(hipMemcpyAsync(occ_offs, q.occ_offs.p, (P + 1) * 8, hipMemcpyDeviceToHost, s));
    if (pos_out && cap >= tot && tot) HK_HIP(hipMemcpyAsync(pos_out, q.pos.p, tot * 8, hipMemcpyDeviceToHost, s));
    HK_HIP(hipStreamSynchronize(s));
    q.trim();
    need(!pos_out || cap >= tot, HKCSA_E_RANGE, "position buffer too small (occ_offs holds the sizes)");
  });
}

// ------------------------------------------------------------ sharded SA
int hkcsa_build_sa_sharded(hkcsa_index* h, const uint8_t id[128], int nranks, int rank) {
  return guarded([&] {
    activate(h);
    need(h->ix.have_text, HKCSA_E_STATE, "text released by hkcsa_compact");
    need(id != nullptr && nranks >= 1 && rank >= 0 && rank < nranks, HKCSA_E_INVALID, "bad communicator args");
    h->ix.have_bwt = h->ix.have_wt = false;
    hk::build_sa_sharded(h->ix, id, nranks, rank);
  });
}

int hkcsa_comm_unique_id(uint8_t id[128]) {
  return guarded([&] {
    need(id != nullptr, HKCSA_E_INVALID, "null output");
    hk::comm_unique_id(id);
  });
}

int hkcsa_shard_buckets(void) { return hk::shard_buckets(); }
int hkcsa_shard_sample(void) { return hk::shard_sample(); }

int hkcsa_shard_scheme(hkcsa_index* h, int* scheme) {
  return guarded([&] {
    activate(h);
    need(scheme != nullptr, HKCSA_E_INVALID, "null output");
    need(h->ix.have_text, HKCSA_E_STATE, "text released by hkcsa_compact");
    *scheme = hk::shard_keyed(h->ix) ? 1 : 0;   // (a query: the alphabet is computed once, if missing)
  });
}

int hkcsa_slice_bounds(const uint64_t* hist, uint32_t nbins, int nslices, uint64_t* below_out) {
  return guarded([&] {
    need(hist != nullptr && below_out != nullptr, HKCSA_E_INVALID, "null buffer");
    need(nbins >= 1 && nbins <= (1u << 24), HKCSA_E_INVALID, "1 to 2^24 bins");
    need(nslices >= 1 && nslices <= 64, HKCSA_E_INVALID, "1 to 64 slices");
    const std::vector<uint64_t> b = hk::slice_bounds(hist, (int)nbins, nslices);
    std::copy(b.begin(), b.end(), below_out);
  });
}

int hkcsa_shard_histogram(hkcsa_index* h, int nranks, int rank, uint64_t* hist_out) {
  return guarded([&] {
    activate(h);
    need(h->ix.have_text, HKCSA_E_STATE, "text released by hkcsa_compact");
    need(hist_out != nullptr && nranks >= 1 && rank >= 0 && rank < nranks, HKCSA_E_INVALID, "bad arguments");
    h->ix.have_alpha = false;   // phase 1 of a build: recompute the byte histogram
    const int nb = hk::shard_buckets();
    hk::DevBuf d;
    d.ensure((size_t)nb * 8);
    hk::shard_histogram(h->ix, nranks, rank, d.as<uint64_t>());
    HK_HIP(hipMemcpyAsync(hist_out, d.p, (size_t)nb * 8, hipMemcpyDeviceToHost, h->ix.stream));
    HK_HIP(hipStreamSynchronize(h->ix.stream));
  });
}

int hkcsa_shard_counts(hkcsa_index* h, const uint64_t* global_hist, int nranks, int rank, uint64_t* below_out) {
  return guarded([&] {
    activate(h);
    need(h->ix.have_text, HKCSA_E_STATE, "text released by hkcsa_compact");
    need(global_hist && below_out && nranks >= 1 && nranks <= 64 && rank >= 0 && rank < nranks, HKCSA_E_INVALID,
         "bad arguments");
    hk::DevBuf d;
    d.ensure((size_t)(nranks + 1) * 8);
    hk::shard_counts(h->ix, global_hist, nranks, rank, d.as<uint64_t>());
    HK_HIP(hipMemcpyAsync(below_out, d.p, (size_t)(nranks + 1) * 8, hipMemcpyDeviceToHost, h->ix.stream));
    HK_HIP(hipStreamSynchronize(h->ix.stream));
  });
}

int hkcsa_shard_build(hkcsa_index* h, const uint64_t* global_hist, const uint64_t* global_below, int nranks,
                      int rank) {
  return guarded([&] {
    activate(h);
    need(h->ix.have_text, HKCSA_E_STATE, "text released by hkcsa_compact");
    need(global_hist && global_below && nranks >= 1 && nranks <= 64 && rank >= 0 && rank < nranks,
         HKCSA_E_INVALID, "bad arguments");
    h->ix.have_bwt = h->ix.have_wt = false;
    hk::shard_build(h->ix, global_hist, global_below, nranks, rank);
  });
}

int hkcsa_get_shard_sa(hkcsa_index* h, uint64_t a, uint64_t b, uint64_t* out) {
  return guarded([&] {
    activate(h);
    need(h->ix.sharded && (h->ix.have_sa || h->ix.dbl.pending), HKCSA_E_STATE, "no sharded suffix array");
    need(a == b || out != nullptr, HKCSA_E_INVALID, "null output");
    hk::shard_get_sa(h->ix, a, b, out);
  });
}

int hkcsa_get_shard_bwt(hkcsa_index* h, uint64_t a, uint64_t b, uint8_t* out) {
  return guarded([&] {
    activate(h);
    need(h->ix.sharded && h->ix.have_bwt, HKCSA_E_STATE, "no sharded BWT");
    need(a == b || out != nullptr, HKCSA_E_INVALID, "null output");
    hk::shard_get_bwt(h->ix, a, b, out);
  });
}

int hkcsa_shard_replicate(hkcsa_index* h) {
  return guarded([&] {
    activate(h);
    hk::shard_replicate(h->ix);
  });
}

int hkcsa_shard_adopt(hkcsa_index* h, const uint64_t* sa, const uint8_t* bwt) {
  return guarded([&] {
    activate(h);
    need(sa && bwt, HKCSA_E_INVALID, "null argument");
    need(h->ix.have_text, HKCSA_E_STATE, "text released by hkcsa_compact");
    need(h->ix.sharded, HKCSA_E_STATE, "adopt: the handle holds no sharded build");
    hk::shard_adopt(h->ix, sa, bwt);   // checks the replica on the GPU (permutation, BWT rows)
  });
}

int hkcsa_shard_status(hkcsa_index* h, uint64_t st[4]) {
  return guarded([&] {
    need(h && st, HKCSA_E_INVALID, "null argument");
    hk::shard_status(h->ix, st);
  });
}

int hkcsa_shard_isa_segment(hkcsa_index* h, const uint64_t* sa, uint64_t count, uint64_t lo) {
  return guarded([&] {
    activate(h);
    need(count == 0 || sa != nullptr, HKCSA_E_INVALID, "null argument");
    hk::shard_isa_segment_host(h->ix, sa, count, lo);
  });
}

int hkcsa_shard_updates(hkcsa_index* h, uint64_t* pairs, uint64_t cap, uint64_t* count) {
  return guarded([&] {
    activate(h);
    need(count != nullptr, HKCSA_E_INVALID, "null argument");
    *count = hk::shard_updates(h->ix, pairs, cap);
  });
}

int hkcsa_shard_apply(hkcsa_index* h, const uint64_t* pairs, uint64_t count) {
  return guarded([&] {
    activate(h);
    need(count == 0 || pairs != nullptr, HKCSA_E_INVALID, "null argument");
    hk::shard_apply_host(h->ix, pairs, count);
  });
}

int hkcsa_shard_round(hkcsa_index* h, uint64_t K) {
  return guarded([&] {
    activate(h);
    hk::shard_round(h->ix, K);
  });
}

int hkcsa_shard_range(hkcsa_index* h, uint64_t* lo, uint64_t* hi) {
  return guarded([&] {
    need(h && lo && hi, HKCSA_E_INVALID, "null argument");
    need(h->ix.sharded, HKCSA_E_STATE, "index is not sharded");
    *lo = h->ix.shard_lo;
    *hi = h->ix.shard_hi;
  });
}

int hkcsa_key_geometry(hkcsa_index* h, int* q, int* pb, uint64_t* radix, int* key_bits) {
  return guarded([&] {
    activate(h);
    need(q && pb && radix && key_bits, HKCSA_E_INVALID, "null output");
    hk::KeyGeom kg = hk::key_geometry(h->ix, true);
    *q = kg.q;
    *pb = kg.pb;
    *radix = kg.R;
    *key_bits = kg.key_bits;
  });
}

// ------------------------------------------------------------ diagnostics
int hkcsa_debug_radix_bench(uint64_t n, int reps, double* out, int nout) {
  return guarded([&] {
    need(out != nullptr && n >= (1u << 16) && reps >= 1, HKCSA_E_INVALID, "bad arguments");
    hk::Index ix;
    init_index(ix, nullptr, n);
    const uint8_t dna[4] = {'A', 'C', 'G', 'T'};
    hk::synth_text(ix.text.as<uint8_t>(), n, dna, 4, 77, '$', ix.stream);
    hk::KeyGeom kg = hk::key_geometry(ix, true);
    hk::upload_geometry(ix, kg);
    for (int i = 0; i < 2; ++i) {
      ix.keys[i].ensure(n * 8 + 16);
      ix.vals[i].ensure(n * 4 + 16);
    }
    hk::pack_keys(ix.text.as<uint8_t>(), n, 0, n, reinterpret_cast<const uint16_t*>(ix.small.as<uint8_t>() + 2048),
                  kg.R, kg.q, kg.pb, ix.keys[0].as<uint64_t>(), ix.stream);
    hk::fill_iota<uint32_t>(ix.vals[0].as<uint32_t>(), n, ix.stream);
    uint64_t* kp[2] = {ix.keys[0].as<uint64_t>(), ix.keys[1].as<uint64_t>()};
    uint32_t* vp[2] = {ix.vals[0].as<uint32_t>(), ix.vals[1].as<uint32_t>()};
    hk::debug_radix_bench(ix.sw, kp, vp, n, kg.pb, reps, out, nout, ix.stream);
    HK_HIP(hipStreamSynchronize(ix.stream));
    (void)hipStreamDestroy(ix.stream);
    ix.stream = nullptr;
  });
}

// ------------------------------------------------------------ timing
int hkcsa_timing_enable(hkcsa_index* h, int on) {
  return guarded([&] {
    activate(h);
    h->ix.timer.resolve();
    h->ix.timer.enabled = on != 0;
  });
}
int hkcsa_timing_reset(hkcsa_index* h) {
  return guarded([&] {
    activate(h);
    h->ix.timer.reset();
  });
}
int hkcsa_kernel_stats(hkcsa_index* h, const char* name, uint64_t* launches, double* total_ms, double* alg_bytes) {
  return guarded([&] {
    activate(h);
    need(name != nullptr, HKCSA_E_INVALID, "null name");
    h->ix.timer.resolve();
    uint64_t l = 0;
    double ms = 0, b = 0;
    for (auto& s : h->ix.timer.stats)
      if (s.first == name) {
        l += s.second.launches;
        ms += s.second.ms;
        b += s.second.bytes;
      }
    if (launches) *launches = l;
    if (total_ms) *total_ms = ms;
    if (alg_bytes) *alg_bytes = b;
  });
}
int hkcsa_build_info(hkcsa_index* h, uint64_t* info, int cap) {
  return guarded([&] {
    need(h && info && cap >= 0, HKCSA_E_INVALID, "null argument");
    const auto& v = h->ix.info;
    for (int i = 0; i < cap; ++i) info[i] = i < (int)v.size() ? v[i] : 0;
  });
}

}  // extern "C"
