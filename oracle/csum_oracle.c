/*
 * csum_oracle.c — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT.
 *
 * CPU restatement of TULIPS' Internet/TCP one's-complement checksum path,
 * written from the reference's behaviour (not copied), used as the parity
 * checker for the HIP kernels and as the "port" CPU baseline in bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this file's shared object (oracle/liboracle.so).
 *
 * Parity pinning: this restatement is checked (tests/test_oracle.py) against
 *   - the known-answer vectors in tests/golden/kat.json, and
 *   - batch digests in tests/golden/digests.json,
 * both produced by tests/golden/make_golden.py from oracle/_ref/libtulips_ref.so,
 * which is the reference's OWN src/stack sources compiled by oracle/Makefile.
 *
 * Reference anchors (paths relative to xenogenics/tulips @ 2024-12-20):
 *   a1 utils::checksum ............ src/stack/Utils.cpp:14-42
 *   a2 tcpv4::Processor::checksum . src/stack/tcpv4/Processor.cpp:337-357
 *   a5 ipv4::checksum ............. src/stack/IPv4.cpp:75-82
 *   a6 icmpv4::checksum ........... src/stack/ICMPv4.cpp:10-15
 * Golden data spec (SplitMix64 arena, Zipf lengths, FNV-1a digest): SURVEY.md §8c.
 */
#include <math.h>
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* Mode numbers shared with include/tulips_csum.h (kept numerically equal). */
#define ORC_MODE_RAW 0u  /* a1 value                                   */
#define ORC_MODE_INET 1u /* a5/a6 post-processing: 0 -> 0xffff, htons  */
#define ORC_MODE_TCP 2u  /* a2: pseudo-header seed + INET post         */
#define ORC_MODE_MASK 0xffu
#define ORC_FLAG_COMPLEMENT 0x100u /* store ~value (generate side)    */

static inline uint16_t orc_bswap16(uint16_t v)
{
  return (uint16_t)((v << 8) | (v >> 8));
}

/*
 * a1 — src/stack/Utils.cpp:14-42. Same loop shape as the reference: a 16-bit
 * accumulator, big-endian byte pairs, carry detected by unsigned wrap and
 * folded back in (:23-30); a trailing odd byte enters as the high byte
 * (:31-37). len == 0 returns the seed unchanged (the reference compares
 * data+len-1 against data and never enters either branch).
 */
uint16_t orc_checksum(uint16_t seed, const uint8_t* data, uint16_t len)
{
  uint16_t acc = seed;
  size_t pairs = (size_t)len / 2u;
  const uint8_t* p = data;
  for (size_t i = 0; i < pairs; ++i, p += 2) {
    uint16_t word = (uint16_t)(((unsigned)p[0] << 8) | (unsigned)p[1]);
    acc = (uint16_t)(acc + word);
    if (acc < word) {
      acc = (uint16_t)(acc + 1u);
    }
  }
  if (len & 1u) {
    uint16_t word = (uint16_t)((unsigned)p[0] << 8);
    acc = (uint16_t)(acc + word);
    if (acc < word) {
      acc = (uint16_t)(acc + 1u);
    }
  }
  return acc;
}

/* Post-processing shared by a2/a5/a6: `sum == 0 ? 0xffff : htons(sum)`
 * (src/stack/IPv4.cpp:80, src/stack/ICMPv4.cpp:14,
 *  src/stack/tcpv4/Processor.cpp:356). Host is little-endian x86. */
static inline uint16_t orc_inet_post(uint16_t sum)
{
  return sum == 0 ? (uint16_t)0xffff : orc_bswap16(sum);
}

/* a5 — src/stack/IPv4.cpp:75-82: a1 over the 20-byte IPv4 header. */
uint16_t orc_ipv4_checksum(const uint8_t* hdr)
{
  return orc_inet_post(orc_checksum(0, hdr, 20));
}

/* a6 — src/stack/ICMPv4.cpp:10-15: a1 over the 8-byte ICMP header ONLY. */
uint16_t orc_icmpv4_checksum(const uint8_t* hdr)
{
  return orc_inet_post(orc_checksum(0, hdr, 8));
}

/*
 * Pseudo-header seed of a2 — src/stack/tcpv4/Processor.cpp:346-351:
 * `sum = len + 6` in uint16 arithmetic (wraps for len > 65529), then a1 over
 * the 4 raw (network-order) bytes of the source address, then of the
 * destination address. `src`/`dst` are the ipv4::Address::m_data words, i.e.
 * the 4 wire bytes read as a native uint32 (include/tulips/stack/IPv4.h:55).
 */
uint16_t orc_tcp_seed(uint32_t src, uint32_t dst, uint16_t len)
{
  uint8_t sb[4], db[4];
  memcpy(sb, &src, 4);
  memcpy(db, &dst, 4);
  uint16_t sum = (uint16_t)(len + 6u);
  sum = orc_checksum(sum, sb, 4);
  sum = orc_checksum(sum, db, 4);
  return sum;
}

/* a2 — src/stack/tcpv4/Processor.cpp:337-357. */
uint16_t orc_tcp_checksum(uint32_t src, uint32_t dst, uint16_t len,
                          const uint8_t* data)
{
  uint16_t sum = orc_checksum(orc_tcp_seed(src, dst, len), data, len);
  return orc_inet_post(sum);
}

/* One segment of a batch, in the same mode/flag vocabulary as the product. */
static inline uint16_t orc_one(const uint8_t* seg, uint16_t len, uint16_t seed,
                               uint32_t src, uint32_t dst, uint32_t mode)
{
  uint16_t v;
  switch (mode & ORC_MODE_MASK) {
    case ORC_MODE_TCP:
      v = orc_inet_post(orc_checksum(orc_tcp_seed(src, dst, len), seg, len));
      break;
    case ORC_MODE_INET:
      v = orc_inet_post(orc_checksum(seed, seg, len));
      break;
    default:
      v = orc_checksum(seed, seg, len);
      break;
  }
  if (mode & ORC_FLAG_COMPLEMENT) {
    v = (uint16_t)~v;
  }
  return v;
}

/*
 * Batch over a packed arena. offsets/lengths describe segment i as
 * base[offsets[i] .. offsets[i]+lengths[i]). When offsets is NULL the
 * segments are at i*stride with the fixed length `fixed_len`.
 * seeds/src/dst may be NULL (seed 0 / address 0).
 */
typedef struct {
  const uint8_t* base;
  const uint64_t* offsets;
  const uint16_t* lengths;
  uint64_t stride;
  uint16_t fixed_len;
  const uint16_t* seeds;
  const uint32_t* src;
  const uint32_t* dst;
  uint16_t* out;
  uint64_t lo, hi;
  uint32_t mode;
} orc_job;

static void orc_run(const orc_job* j)
{
  for (uint64_t i = j->lo; i < j->hi; ++i) {
    uint64_t off = j->offsets ? j->offsets[i] : i * j->stride;
    uint16_t len = j->lengths ? j->lengths[i] : j->fixed_len;
    j->out[i] = orc_one(j->base + off, len, j->seeds ? j->seeds[i] : 0,
                        j->src ? j->src[i] : 0, j->dst ? j->dst[i] : 0,
                        j->mode);
  }
}

static void* orc_thread(void* arg)
{
  orc_run((const orc_job*)arg);
  return NULL;
}

/* Returns 0 on success, -1 on bad arguments / thread failure. */
int orc_batch(const uint8_t* base, const uint64_t* offsets,
              const uint16_t* lengths, uint64_t stride, uint32_t fixed_len,
              const uint16_t* seeds, const uint32_t* src, const uint32_t* dst,
              uint16_t* out, uint64_t n, uint32_t mode, int nthreads)
{
  if (fixed_len > 0xffffu || (n && (!base || !out))) {
    return -1;
  }
  if ((mode & ORC_MODE_MASK) > ORC_MODE_TCP) {
    return -1;
  }
  if (nthreads < 1) {
    nthreads = 1;
  }
  if ((uint64_t)nthreads > n) {
    nthreads = n ? (int)n : 1;
  }
  orc_job jobs[256];
  pthread_t tids[256];
  if (nthreads > 256) {
    nthreads = 256;
  }
  for (int t = 0; t < nthreads; ++t) {
    orc_job* j = &jobs[t];
    j->base = base;
    j->offsets = offsets;
    j->lengths = lengths;
    j->stride = stride;
    j->fixed_len = (uint16_t)fixed_len;
    j->seeds = seeds;
    j->src = src;
    j->dst = dst;
    j->out = out;
    j->lo = n * (uint64_t)t / (uint64_t)nthreads;
    j->hi = n * (uint64_t)(t + 1) / (uint64_t)nthreads;
    j->mode = mode;
  }
  if (nthreads == 1) {
    orc_run(&jobs[0]);
    return 0;
  }
  int rc = 0, started = 0;
  for (int t = 0; t < nthreads; ++t, ++started) {
    if (pthread_create(&tids[t], NULL, orc_thread, &jobs[t]) != 0) {
      rc = -1;
      break;
    }
  }
  for (int t = 0; t < started; ++t) {
    pthread_join(tids[t], NULL);
  }
  return rc;
}

/* ---------------------------------------------------------------------------
 * Golden-data generators (SURVEY.md §8c "Golden batch spec").
 * ------------------------------------------------------------------------- */

static inline uint64_t orc_splitmix_mix(uint64_t z)
{
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/*
 * Arena bytes [byte_off, byte_off+nbytes) of the SplitMix64 stream with
 * state `seed`: draw k (k = 0,1,...) is mix(seed + (k+1)*golden) and
 * supplies arena bytes 8k..8k+7 little-endian.
 */
void orc_fill_splitmix(uint8_t* dst, uint64_t nbytes, uint64_t seed,
                       uint64_t byte_off)
{
  for (uint64_t i = 0; i < nbytes;) {
    uint64_t b = byte_off + i;
    uint64_t k = b >> 3;
    uint64_t z = orc_splitmix_mix(seed + (k + 1) * 0x9E3779B97F4A7C15ull);
    unsigned sh = (unsigned)(b & 7u);
    for (; sh < 8 && i < nbytes; ++sh, ++i) {
      dst[i] = (uint8_t)(z >> (8 * sh));
    }
  }
}

/*
 * Zipf segment lengths: u = (next()>>11)*2^-53 from SplitMix64(seed),
 * C[r] = sum_{k<=r} k^-1.1 for r = 1..rmax, r = first index with
 * C[r] >= u*C[rmax], length = 63 + r.
 */
int orc_zipf_lengths(uint16_t* out, uint64_t n, uint64_t seed, uint32_t rmax)
{
  if (rmax == 0 || rmax > 65535u - 63u) {
    return -1;
  }
  double* c = (double*)malloc(sizeof(double) * (rmax + 1));
  if (!c) {
    return -1;
  }
  c[0] = 0.0;
  for (uint32_t r = 1; r <= rmax; ++r) {
    c[r] = c[r - 1] + pow((double)r, -1.1);
  }
  uint64_t s = seed;
  for (uint64_t i = 0; i < n; ++i) {
    s += 0x9E3779B97F4A7C15ull;
    double u = (double)(orc_splitmix_mix(s) >> 11) * 0x1.0p-53;
    double target = u * c[rmax];
    uint32_t lo = 1, hi = rmax; /* first r with c[r] >= target */
    while (lo < hi) {
      uint32_t mid = lo + (hi - lo) / 2;
      if (c[mid] >= target) {
        hi = mid;
      } else {
        lo = mid + 1;
      }
    }
    out[i] = (uint16_t)(63u + lo);
  }
  free(c);
  return 0;
}

/* FNV-1a-64 over each u16 as 2 little-endian bytes, in order. */
uint64_t orc_fnv1a_u16(const uint16_t* v, uint64_t n)
{
  uint64_t h = 0xcbf29ce484222325ull;
  for (uint64_t i = 0; i < n; ++i) {
    h ^= (uint64_t)(v[i] & 0xffu);
    h *= 0x100000001b3ull;
    h ^= (uint64_t)(v[i] >> 8);
    h *= 0x100000001b3ull;
  }
  return h;
}

uint64_t orc_sum_u16(const uint16_t* v, uint64_t n)
{
  uint64_t s = 0;
  for (uint64_t i = 0; i < n; ++i) {
    s += v[i];
  }
  return s;
}

/* ---------------------------------------------------------------------------
 * §8f #3 — Toeplitz RSS hash, src/stack/Utils.cpp:86-133 (restated).
 * tuple = saddr bytes | daddr bytes | htons(sport) | htons(dport) (:101-111);
 * for each tuple bit MSB first, XOR the big-endian first 4 key bytes into the
 * hash when the bit is set (:117-119), then shift the key left by one bit with
 * the reference's wrap-around, which reads the ALREADY-SHIFTED tmp[0] for the
 * last byte (:123-125). Keys shorter than 4 bytes are rejected (the reference
 * reads 4 bytes of the key buffer whatever its length).
 * ------------------------------------------------------------------------- */
int orc_toeplitz(uint32_t saddr, uint32_t daddr, uint16_t sport, uint16_t dport,
                 size_t len, const uint8_t* key, uint32_t init, uint32_t* out)
{
  if (len < 4 || len > 1024 || !key || !out) {
    return -1;
  }
  uint8_t tmp[1024], tuple[12];
  memcpy(tmp, key, len);
  memcpy(tuple, &saddr, 4);
  memcpy(tuple + 4, &daddr, 4);
  tuple[8] = (uint8_t)(sport >> 8);
  tuple[9] = (uint8_t)sport;
  tuple[10] = (uint8_t)(dport >> 8);
  tuple[11] = (uint8_t)dport;
  uint32_t h = init;
  for (int b = 0; b < 12; ++b) {
    for (int j = 0; j < 8; ++j) {
      if (tuple[b] & (1u << (7 - j))) {
        h ^= ((uint32_t)tmp[0] << 24) | ((uint32_t)tmp[1] << 16) |
             ((uint32_t)tmp[2] << 8) | (uint32_t)tmp[3];
      }
      for (size_t i = 0; i < len; ++i) {
        tmp[i] = (uint8_t)(((tmp[i] << 1) & 0xff) | ((tmp[(i + 1) % len] & 0x80) >> 7));
      }
    }
  }
  *out = h;
  return 0;
}

/* ---------------------------------------------------------------------------
 * §8f #1/#2 — receive-side validation of one Ethernet frame, restating the
 * checks the stack applies before a segment reaches TCP:
 *   ethernet/Processor.cpp:69,91      type 0x0800 -> IPv4
 *   ipv4/Processor.cpp:67-73          vhl must be 0x45
 *   ipv4/Processor.cpp:77-82          no fragments
 *   ipv4/Processor.cpp:94-103         ipv4::checksum(header) == 0xffff
 *   ipv4/Processor.cpp:108,116-122    proto 6 -> TCP over ntohs(len) - 20 bytes
 *   tcpv4/Processor.cpp:121-131       tcpv4 checksum == 0xffff
 * The destination-address filter (ipv4/Processor.cpp:86-92) is the caller's.
 * Flags (numerically equal to TULIPS_FRAME_* in include/tulips_csum.h):
 * ------------------------------------------------------------------------- */
#define ORC_FRAME_IPV4 0x01u
#define ORC_FRAME_IP_CSUM_OK 0x02u
#define ORC_FRAME_TCP 0x04u
#define ORC_FRAME_L4_CSUM_OK 0x08u
#define ORC_FRAME_TRUNCATED 0x10u

uint8_t orc_validate_frame(const uint8_t* f, uint32_t len)
{
  if (len < 14 || ((unsigned)f[12] << 8 | f[13]) != 0x0800u) {
    return 0;
  }
  if (len < 34) {
    return ORC_FRAME_TRUNCATED;
  }
  const uint8_t* ip = f + 14;
  if (ip[0] != 0x45) {
    return 0;
  }
  uint8_t fl = ORC_FRAME_IPV4;
  if (orc_ipv4_checksum(ip) == 0xffff) {
    fl |= ORC_FRAME_IP_CSUM_OK;
  }
  if ((ip[6] & 0x3f) != 0 || ip[7] != 0 || ip[9] != 6) {
    return fl;
  }
  fl |= ORC_FRAME_TCP;
  const uint16_t total = (uint16_t)((ip[2] << 8) | ip[3]);
  const uint16_t tcplen = (uint16_t)(total - 20u);
  if (total < 20 || 34u + tcplen > len) {
    return (uint8_t)(fl | ORC_FRAME_TRUNCATED);
  }
  uint32_t src, dst;
  memcpy(&src, ip + 12, 4);
  memcpy(&dst, ip + 16, 4);
  if (orc_tcp_checksum(src, dst, tcplen, ip + 20) == 0xffff) {
    fl |= ORC_FRAME_L4_CSUM_OK;
  }
  return fl;
}

void orc_validate_frames(const uint8_t* base, const uint64_t* offsets,
                         const uint16_t* lengths, uint64_t n, uint8_t* flags)
{
  for (uint64_t i = 0; i < n; ++i) {
    flags[i] = orc_validate_frame(base + offsets[i], lengths[i]);
  }
}

/* ---------------------------------------------------------------------------
 * §8f #4 — send-side checksum generation of one frame, in place:
 *   ipv4/Producer.cpp:79-82   ipchksum = 0; ipchksum = ~ipv4::checksum(hdr)
 *   tcpv4/Send.cpp:441-449    chksum = 0;   chksum = ~checksum(src, dst, len, seg)
 * applied to option-less IPv4 frames and unfragmented TCP ones whose
 * ntohs(len) - 20 byte segment (>= 18 bytes, so the field exists) fits.
 * Returns the TULIPS_FRAME_* bits: IP_CSUM_OK / L4_CSUM_OK = field written.
 * ------------------------------------------------------------------------- */
uint8_t orc_generate_frame(uint8_t* f, uint32_t len)
{
  if (len < 14 || ((unsigned)f[12] << 8 | f[13]) != 0x0800u) {
    return 0;
  }
  if (len < 34) {
    return ORC_FRAME_TRUNCATED;
  }
  uint8_t* ip = f + 14;
  if (ip[0] != 0x45) {
    return 0;
  }
  ip[10] = ip[11] = 0;
  uint16_t c = (uint16_t)~orc_ipv4_checksum(ip);
  memcpy(ip + 10, &c, 2);
  uint8_t fl = ORC_FRAME_IPV4 | ORC_FRAME_IP_CSUM_OK;
  if ((ip[6] & 0x3f) != 0 || ip[7] != 0 || ip[9] != 6) {
    return fl;
  }
  fl |= ORC_FRAME_TCP;
  const uint16_t total = (uint16_t)((ip[2] << 8) | ip[3]);
  const uint16_t tcplen = (uint16_t)(total - 20u);
  if (total < 20 || 34u + tcplen > len) {
    return (uint8_t)(fl | ORC_FRAME_TRUNCATED);
  }
  if (tcplen < 18) {
    return fl;
  }
  uint32_t src, dst;
  memcpy(&src, ip + 12, 4);
  memcpy(&dst, ip + 16, 4);
  ip[36] = ip[37] = 0;
  c = (uint16_t)~orc_tcp_checksum(src, dst, tcplen, ip + 20);
  memcpy(ip + 36, &c, 2);
  return (uint8_t)(fl | ORC_FRAME_L4_CSUM_OK);
}

void orc_generate_frames(uint8_t* base, const uint64_t* offsets,
                         const uint16_t* lengths, uint64_t n, uint8_t* flags)
{
  for (uint64_t i = 0; i < n; ++i) {
    const uint8_t fl = orc_generate_frame(base + offsets[i], lengths[i]);
    if (flags) {
      flags[i] = fl;
    }
  }
}

/* ---------------------------------------------------------------------------
 * §8f #4 — segmentation offload (the NIC's side of IBV_WR_TSO,
 * src/transport/ofed/Device.cpp:688-772; header length as
 * stack::utils::headerLength, src/stack/Utils.cpp:67-84). Standard LSO
 * fixups (PARITY UNPINNED: the reference has no software TSO) followed by
 * orc_generate_frame, which is pinned to the reference's generation.
 * ------------------------------------------------------------------------- */
static uint32_t orc_seg_count(const uint8_t* f, uint32_t len, uint32_t mss,
                              int* seg_ok, uint32_t* hlen, uint32_t* payload)
{
  *seg_ok = 0;
  *hlen = 0;
  *payload = 0;
  const uint8_t fl = orc_validate_frame(f, len);
  if (!(fl & ORC_FRAME_TCP) || (fl & ORC_FRAME_TRUNCATED)) {
    return 1;
  }
  const uint32_t doff = len > 46 ? (uint32_t)(f[46] >> 4) : 0u;
  const uint32_t total = (uint32_t)(f[16] << 8 | f[17]);
  if (doff < 5 || 20u + 4u * doff > total) {
    return 1;
  }
  *seg_ok = 1;
  *hlen = 34u + 4u * doff;
  *payload = total - 20u - 4u * doff;
  return *payload > mss ? (*payload + mss - 1) / mss : 1u;
}

/* first[] gets n + 1 entries; returns the total number of segments. */
uint32_t orc_segment_count(const uint8_t* base, const uint64_t* offsets,
                           const uint16_t* lengths, uint32_t n, uint32_t mss,
                           uint32_t* first)
{
  uint32_t acc = 0;
  for (uint32_t i = 0; i < n; ++i) {
    int ok;
    uint32_t h, p;
    first[i] = acc;
    acc += orc_seg_count(base + offsets[i], lengths[i], mss, &ok, &h, &p);
  }
  first[n] = acc;
  return acc;
}

void orc_segment_frames(const uint8_t* base, const uint64_t* offsets,
                        const uint16_t* lengths, uint32_t n, uint32_t mss,
                        uint8_t* out, uint64_t stride, uint32_t capacity,
                        uint16_t* out_lengths, const uint32_t* first)
{
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t* f = base + offsets[i];
    const uint32_t len = lengths[i];
    int ok;
    uint32_t hlen, payload;
    const uint32_t nseg = orc_seg_count(f, len, mss, &ok, &hlen, &payload);
    for (uint32_t k = 0; k < nseg; ++k) {
      const uint32_t j = first[i] + k;
      if (j >= capacity) {
        break;
      }
      uint8_t* d = out + (uint64_t)j * stride;
      if (nseg == 1) {
        if (len > stride) {
          out_lengths[j] = 0;
          continue;
        }
        memcpy(d, f, len);
        orc_generate_frame(d, len);
        out_lengths[j] = (uint16_t)len;
        continue;
      }
      const uint32_t slice = payload - k * mss < mss ? payload - k * mss : mss;
      const uint32_t dlen = hlen + slice;
      if (dlen > stride) {
        out_lengths[j] = 0;
        continue;
      }
      memcpy(d, f, hlen);
      memcpy(d + hlen, f + hlen + (uint64_t)k * mss, slice);
      const uint32_t total = dlen - 14u;
      d[16] = (uint8_t)(total >> 8);
      d[17] = (uint8_t)total;
      const uint32_t id = ((uint32_t)(f[18] << 8 | f[19]) + k) & 0xffffu;
      d[18] = (uint8_t)(id >> 8);
      d[19] = (uint8_t)id;
      const uint32_t seq = ((uint32_t)f[38] << 24 | (uint32_t)f[39] << 16 |
                            (uint32_t)f[40] << 8 | f[41]) + k * mss;
      d[38] = (uint8_t)(seq >> 24);
      d[39] = (uint8_t)(seq >> 16);
      d[40] = (uint8_t)(seq >> 8);
      d[41] = (uint8_t)seq;
      uint8_t tfl = f[47];
      if (k + 1 < nseg) {
        tfl &= (uint8_t)~(0x01 | 0x08); /* FIN, PSH on the last segment only */
      }
      if (k > 0) {
        tfl &= (uint8_t)~0x80; /* CWR on the first segment only */
      }
      d[47] = tfl;
      orc_generate_frame(d, dlen);
      out_lengths[j] = (uint16_t)dlen;
    }
  }
}
