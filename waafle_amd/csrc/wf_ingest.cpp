// Native ingest of the waafle_orgscorer inputs: FASTA lengths,
// BLAST tabular hits and GFF loci parsed into the CSR arrays wf_score() takes.
//
// Restates, for well-formed input, waafle/utils.py:109-120 (read_contig_lengths),
// :207-241 + :255-270 (Hit, iter_contig_hits), :300-322 + :341-355 (Locus,
// iter_contig_loci) and waafle/waafle_orgscorer.py:348-357, 908-946 (locus length filter,
// FASTA-ordered contigs, unknown-contig warnings).  The Python restatement of the same
// readers is waafle_amd/inputs.py; any input outside the plain spelling this parser
// accepts (see include/waafle_ingest.h) returns WF_INGEST_FALLBACK so that reader decides.
//
// Layout of the work: the BLAST file (by far the largest) is memory-mapped and cut into
// one chunk per thread at line boundaries.  Each thread parses its rows into a local
// record array and interns taxa / annotation strings locally.  A serial pass groups rows
// by consecutive qseqid (utils.py:262-266) and maps groups to FASTA contigs; a second
// parallel pass gathers the kept rows into FASTA contig order and derives scov_modified
// and waafle_score with the reference's float64 operations in the reference's order.
#include "waafle_ingest.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include <emmintrin.h>

namespace wf_ing {

// Anonymous pages for the large arrays, in transparent huge pages where the kernel allows
// them (MADV_HUGEPAGE): the threads that first touch them fault 2 MB at a time instead of
// 4 KB, which otherwise serialises them on the address-space lock.
void* big_alloc(size_t bytes) {
  if (bytes == 0) bytes = 1;
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
  if (p == MAP_FAILED) throw std::bad_alloc();
#ifdef MADV_HUGEPAGE
  if (bytes >= (2u << 20)) madvise(p, bytes, MADV_HUGEPAGE);
#endif
  return p;
}

template <class T>
struct PodArray {
  T* p = nullptr;
  size_t n = 0, bytes = 0;
  PodArray() = default;
  PodArray(const PodArray&) = delete;
  PodArray& operator=(const PodArray&) = delete;
  PodArray(PodArray&& o) noexcept { *this = std::move(o); }
  PodArray& operator=(PodArray&& o) noexcept {
    if (this != &o) {
      release();
      p = o.p; n = o.n; bytes = o.bytes;
      o.p = nullptr; o.n = o.bytes = 0;
    }
    return *this;
  }
  ~PodArray() { release(); }
  void release() {
    if (p) munmap(p, bytes);
    p = nullptr;
    n = bytes = 0;
  }
  void alloc(size_t count) {
    release();
    bytes = std::max<size_t>(count, 1) * sizeof(T);
    p = static_cast<T*>(big_alloc(bytes));
    n = count;
  }
  T& operator[](size_t i) { return p[i]; }
  const T& operator[](size_t i) const { return p[i]; }
  const T* data() const { return p; }
};

// Append-only array with a fixed capacity reserved up front (virtual; pages are touched as
// rows arrive).  The capacity bounds what one chunk can hold (a BLAST row is >= 30 bytes).
template <class T>
struct Appender {
  PodArray<T> a;
  size_t len = 0;
  void reserve(size_t cap) { a.alloc(cap); len = 0; }
  bool push(const T& x) {
    if (len == a.n) return false;
    a.p[len++] = x;
    return true;
  }
  size_t size() const { return len; }
  const T& operator[](size_t i) const { return a.p[i]; }
};

}  // namespace wf_ing

namespace {

using sv = std::string_view;
using wf_ing::Appender;
using wf_ing::PodArray;

struct Mapped {
  const char* p = nullptr;
  size_t n = 0;
  void* base = nullptr;
  ~Mapped() {
    if (base) munmap(base, n);
  }
  bool open(const char* path, std::string* err) {
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) { *err = std::string("cannot open ") + path; return false; }
    struct stat st;
    if (fstat(fd, &st) != 0) { ::close(fd); *err = std::string("cannot stat ") + path; return false; }
    n = (size_t)st.st_size;
    if (n > 0) {
      base = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
      if (base == MAP_FAILED) { base = nullptr; ::close(fd); *err = std::string("cannot map ") + path; return false; }
      madvise(base, n, MADV_SEQUENTIAL);
      p = static_cast<const char*>(base);
    } else {
      p = "";
    }
    ::close(fd);
    return true;
  }
};

// Bytes that make a file "unusual": a carriage return that is not part of a "\r\n" line end
// (Python's universal newlines would split the line there), bytes >= 0x80 (len() counts
// code points) and NUL (csv rejects it).  Quote characters are plain except at the start
// of a csv field (split_tabs).
bool all_plain(const char* b, const char* e) {
  // NUL or >= 0x80 <=> (uint8)(c - 1) >= 0x7F: a max-reduction the compiler vectorises
  const unsigned char* p = reinterpret_cast<const unsigned char*>(b);
  const size_t n = (size_t)(e - b);
  for (size_t i = 0; i < n;) {
    const size_t m = std::min<size_t>(n - i, 1 << 16);
    unsigned char acc = 0;
    for (size_t j = 0; j < m; ++j) {
      const unsigned char d = (unsigned char)(p[i + j] - 1u);
      acc = d > acc ? d : acc;
    }
    if (acc >= 0x7F) return false;
    i += m;
  }
  for (const char* q = b; (q = static_cast<const char*>(memchr(q, '\r', (size_t)(e - q)))) != nullptr; ++q)
    if (q + 1 < e && q[1] != '\n') return false;
  return true;
}

// End of the line starting at p ('\n' or the end of the file), and the end of its text
// (a "\r\n" or final "\r" line end is not text, as under universal newlines).
inline const char* line_end(const char* p, const char* end, const char** text_end) {
  const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
  const char* le = nl ? nl : end;
  *text_end = (le > p && le[-1] == '\r') ? le - 1 : le;
  return le;
}

// Python str.strip()/split() whitespace within ASCII.
inline bool py_space(unsigned char c) {
  return c == ' ' || (c >= '\t' && c <= '\r') || (c >= 0x1c && c <= 0x1f);
}

// [+-]?[0-9]+ into int64.
// (up to 18 digits; longer spellings go to the Python reader)
bool parse_int(sv f, int64_t& out) {
  size_t i = 0;
  bool neg = false;
  if (i < f.size() && (f[i] == '+' || f[i] == '-')) { neg = f[i] == '-'; ++i; }
  if (i == f.size() || f.size() - i > 18) return false;
  int64_t v = 0;
  for (; i < f.size(); ++i) {
    const unsigned d = (unsigned)(f[i] - '0');
    if (d > 9) return false;
    v = v * 10 + (int64_t)d;
  }
  out = neg ? -v : v;
  return true;
}

// [+-]? (digits [. digits?] | . digits) ([eE] [+-]? digits)?, correctly rounded (same
// result as Python float() / numpy's string conversion).
bool parse_float(sv f, double& out) {
  size_t i = 0;
  bool neg = false;
  if (i < f.size() && (f[i] == '+' || f[i] == '-')) { neg = f[i] == '-'; ++i; }
  const size_t m0 = i;
  size_t nd = 0;
  while (i < f.size() && f[i] >= '0' && f[i] <= '9') { ++i; ++nd; }
  if (i < f.size() && f[i] == '.') {
    ++i;
    while (i < f.size() && f[i] >= '0' && f[i] <= '9') { ++i; ++nd; }
  }
  if (nd == 0) return false;
  if (i < f.size() && (f[i] == 'e' || f[i] == 'E')) {
    ++i;
    if (i < f.size() && (f[i] == '+' || f[i] == '-')) ++i;
    size_t ne = 0;
    while (i < f.size() && f[i] >= '0' && f[i] <= '9') { ++i; ++ne; }
    if (ne == 0) return false;
  }
  if (i != f.size()) return false;
  // Clinger's fast path: a decimal with <= 15 digits and no exponent is M / 10^k with M
  // and 10^k (k <= 22) exact doubles, so one IEEE division is the correctly rounded value
  if (nd <= 15 && (f.size() - m0) <= 16 && f.find_first_of("eE", m0) == sv::npos) {
    static const double p10[] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10,
                                 1e11, 1e12, 1e13, 1e14, 1e15, 1e16};
    uint64_t mant = 0;
    int frac = -1;
    for (size_t j = m0; j < f.size(); ++j) {
      if (f[j] == '.') { frac = 0; continue; }
      mant = mant * 10 + (uint64_t)(f[j] - '0');
      if (frac >= 0) ++frac;
    }
    const double v = (double)mant / p10[frac < 0 ? 0 : frac];
    out = neg ? -v : v;
    return true;
  }
  double v = 0.0;
  const auto r = std::from_chars(f.data() + m0, f.data() + f.size(), v, std::chars_format::general);
  if (r.ec != std::errc() || r.ptr != f.data() + f.size()) return false;
  out = neg ? -v : v;
  return true;
}

// Split a line into exactly N tab-separated fields, as csv's excel-tab dialect does for
// lines without quoting: a field that starts with '"' would be a quoted field, so such a
// line is left to the Python reader (quotes elsewhere in a field are literal in csv).
template <int N>
bool split_tabs(const char* b, const char* e, sv (&f)[N]) {
  int k = 0;
  const char* s = b;
  for (const char* q = b; q < e; ++q) {
    if (*q == '\t') {
      if (k == N - 1 || *s == '"') return false;
      f[k++] = sv(s, (size_t)(q - s));
      s = q + 1;
    }
  }
  if (k != N - 1 || (s < e && *s == '"')) return false;
  f[k] = sv(s, (size_t)(e - s));
  return true;
}

// Hash of a short string: 8-byte words folded by multiply-xor (the texts interned here --
// taxa, annotation systems and values -- are a few to a few dozen bytes).
inline uint64_t text_hash(sv s, uint64_t seed = 0) {
  uint64_t h = seed ^ (0x9E3779B97F4A7C15ull * (s.size() + 1));
  size_t i = 0;
  for (; i + 8 <= s.size(); i += 8) {
    uint64_t w;
    memcpy(&w, s.data() + i, 8);
    h = (h ^ w) * 0xBF58476D1CE4E5B9ull;
    h ^= h >> 31;
  }
  uint64_t w = 0;
  for (size_t j = s.size(); j > i; --j) w = (w << 8) | (unsigned char)s[j - 1];
  h ^= w;                                     // murmur3's 64-bit finaliser
  h = (h ^ (h >> 33)) * 0xFF51AFD7ED558CCDull;
  h = (h ^ (h >> 33)) * 0xC4CEB9FE1A85EC53ull;
  return h ^ (h >> 33);
}

// Open-addressing map from (tag, text) to dense ids 0, 1, ...: no node allocation per
// entry, one probe sequence over a flat table (load factor <= 1/2).  The texts are copied
// into the map's own blocks: a compare then reads cache-resident bytes, not the first
// occurrence's line somewhere in a multi-GB mapping.
struct FlatIds {
  struct Slot { uint64_t h; int32_t id; int32_t tag; };
  std::vector<Slot> tab;
  std::vector<sv> texts;                      // by id (into `blocks`)
  std::vector<std::unique_ptr<char[]>> blocks;
  size_t block_left = 0;
  char* block_at = nullptr;
  size_t mask = 0;
  FlatIds() { tab.assign(1024, Slot{0, -1, 0}); mask = 1023; }
  sv keep(sv s) {
    if (s.size() > block_left) {
      const size_t n = std::max<size_t>(s.size(), 1 << 16);
      blocks.emplace_back(new char[n]);
      block_at = blocks.back().get();
      block_left = n;
    }
    memcpy(block_at, s.data(), s.size());
    const sv out(block_at, s.size());
    block_at += s.size();
    block_left -= s.size();
    return out;
  }
  int32_t get(sv s, int32_t tag = 0) {
    const uint64_t h = text_hash(s, (uint64_t)(uint32_t)tag);
    for (size_t i = (size_t)h & mask;; i = (i + 1) & mask) {
      Slot& e = tab[i];
      if (e.id < 0) {
        const int32_t id = (int32_t)texts.size();
        e = Slot{h, id, tag};
        texts.push_back(keep(s));
        if (texts.size() * 2 > tab.size()) grow();
        return id;
      }
      if (e.h == h && e.tag == tag && texts[e.id] == s) return e.id;
    }
  }
  void grow() {
    std::vector<Slot> old;
    old.swap(tab);
    tab.assign(old.size() * 2, Slot{0, -1, 0});
    mask = tab.size() - 1;
    for (const Slot& e : old) {
      if (e.id < 0) continue;
      size_t i = (size_t)e.h & mask;
      while (tab[i].id >= 0) i = (i + 1) & mask;
      tab[i] = e;
    }
  }
};

struct Interner {
  FlatIds ids;
  std::vector<sv>& names = ids.texts;
  int32_t get(sv s) { return ids.get(s); }
};

// One BLAST row, reduced at parse time to what the hit arrays hold (utils.py:207-241): the
// derived scov_modified / waafle_score are computed here, in the reference's order; a row
// whose derivation fails records why (`bad`), which matters only if the row is kept.
struct Row {
  int32_t qlo, qhi;               // min / max(qstart, qend)
  int32_t taxon;                  // thread-local taxon id (-1: bad sseqid)
  int32_t ann_off;                // thread-local annotation pairs [ann_off, ann_off + ann_n)
  double scov, score;
  int16_t ann_n;
  uint8_t minus;
  uint8_t bad;                    // 0, or 1 slen/qlen 0, 2 denominator 0, 3 q outside int32
};

// Rows of one qseqid in a row: [r0, r1) of a chunk (utils.py:262-266 groups by these)
struct QRun {
  sv q;
  int64_t r0, r1;
};

struct Chunk {
  const char* b;
  const char* e;
  Appender<Row> rows;
  std::vector<QRun> runs;
  Appender<std::pair<int32_t, int32_t>> ann;     // (local system, local value)
  Interner taxa, systems;
  FlatIds values;                                 // (local system, text) -> local value id
  std::vector<int32_t> value_sys;                 // local system of each local value
  sv last_sys;                                    // the previous annotation's system ...
  int32_t last_sys_id = -1;                       // ... and its id (rows repeat systems)
  std::string err;                                // non-empty: fallback
};

// Numeric check of a float field that is only validated (evalue, bitscore): the plain
// spelling parse_float accepts, without the conversion.
bool plain_float(sv f) {
  size_t i = 0;
  if (i < f.size() && (f[i] == '+' || f[i] == '-')) ++i;
  size_t nd = 0;
  while (i < f.size() && f[i] >= '0' && f[i] <= '9') { ++i; ++nd; }
  if (i < f.size() && f[i] == '.') {
    ++i;
    while (i < f.size() && f[i] >= '0' && f[i] <= '9') { ++i; ++nd; }
  }
  if (nd == 0) return false;
  if (i < f.size() && (f[i] == 'e' || f[i] == 'E')) {
    ++i;
    if (i < f.size() && (f[i] == '+' || f[i] == '-')) ++i;
    size_t ne = 0;
    while (i < f.size() && f[i] >= '0' && f[i] <= '9') { ++i; ++ne; }
    if (ne == 0) return false;
  }
  return i == f.size();
}

bool plain_int(sv f) {
  size_t i = 0;
  if (i < f.size() && (f[i] == '+' || f[i] == '-')) ++i;
  if (i == f.size() || f.size() - i > 18) return false;   // (int64 range, as parse_int)
  for (; i < f.size(); ++i)
    if ((unsigned)(f[i] - '0') > 9) return false;
  return true;
}

// One BLAST row (utils.py:207-241).  Numeric columns are validated for every row, as the
// reference converts every field of every row; sseqid problems are recorded and only
// matter for rows of known contigs.
bool parse_blast_row(const sv (&f)[15], Chunk& ck) {
  int64_t qlen, slen, qstart, qend, sstart, send;
  double pident;
  if (!parse_int(f[2], qlen) || !parse_int(f[3], slen) || !plain_int(f[4]) ||
      !parse_int(f[5], qstart) || !parse_int(f[6], qend) || !parse_int(f[7], sstart) ||
      !parse_int(f[8], send) || !plain_int(f[10]) || !plain_int(f[11])) {
    ck.err = "BLAST integer field outside the plain spelling";
    return false;
  }
  if (!parse_float(f[9], pident) || !plain_float(f[12]) || !plain_float(f[13])) {
    ck.err = "BLAST float field outside the plain spelling";
    return false;
  }
  Row r;
  r.minus = f[14] == "minus" ? 1 : 0;
  r.bad = 0;
  r.scov = r.score = 0.0;
  // utils.py:216-229, evaluated as the reference does (int64, then float64)
  if (slen == 0 || qlen == 0) {
    r.bad = 1;
  } else {
    const int64_t s0 = r.minus ? slen - sstart + 1 : sstart;
    const int64_t s1 = r.minus ? slen - send + 1 : send;
    const int64_t ltrim = std::max<int64_t>(0, s0 - qstart);
    const int64_t rtrim = std::max<int64_t>(0, slen - s0 - qlen + qstart);
    const int64_t den = slen - ltrim - rtrim;
    if (den == 0) {
      r.bad = 2;
    } else {
      r.scov = (double)(s1 - s0 + 1) / (double)den;
      r.score = r.scov * pident / 100.0;
    }
  }
  if (qstart < INT32_MIN || qstart > INT32_MAX || qend < INT32_MIN || qend > INT32_MAX) {
    r.bad = r.bad ? r.bad : 3;
    r.qlo = r.qhi = 0;
  } else {
    r.qlo = (int32_t)std::min(qstart, qend);
    r.qhi = (int32_t)std::max(qstart, qend);
  }
  // qseqid runs
  const sv q = f[0];
  const int64_t i = (int64_t)ck.rows.size();
  if (ck.runs.empty() || ck.runs.back().q != q) ck.runs.push_back(QRun{q, i, i});
  ck.runs.back().r1 = i + 1;
  // sseqid: gene | taxon | system=value ... (utils.py:231-241)
  const sv sid = f[1];
  r.taxon = -1;
  if (ck.ann.size() > (size_t)INT32_MAX - 4096) { ck.err = "BLAST chunk annotation count"; return false; }
  r.ann_off = (int32_t)ck.ann.size();
  r.ann_n = 0;
  size_t p1 = sid.find('|');
  if (p1 != sv::npos) {
    size_t p2 = sid.find('|', p1 + 1);
    const sv taxon = sid.substr(p1 + 1, p2 == sv::npos ? sv::npos : p2 - p1 - 1);
    bool ok = true;
    while (p2 != sv::npos) {
      const size_t p3 = sid.find('|', p2 + 1);
      const sv item = sid.substr(p2 + 1, p3 == sv::npos ? sv::npos : p3 - p2 - 1);
      const size_t eq = item.find('=');
      if (eq == sv::npos || item.find('=', eq + 1) != sv::npos || r.ann_n == INT16_MAX) { ok = false; break; }
      const sv sys = item.substr(0, eq), val = item.substr(eq + 1);
      if (ck.last_sys_id < 0 || sys != ck.last_sys) {
        ck.last_sys = sys;
        ck.last_sys_id = ck.systems.get(sys);
      }
      const int32_t s = ck.last_sys_id;
      const int32_t v = ck.values.get(val, s);
      if (v == (int32_t)ck.value_sys.size()) ck.value_sys.push_back(s);   // (a new value)
      if (!ck.ann.push(std::make_pair(s, v))) { ck.err = "BLAST chunk annotation capacity"; return false; }
      ++r.ann_n;
      p2 = p3;
    }
    if (ok) r.taxon = ck.taxa.get(taxon);
  }
  if (!ck.rows.push(r)) { ck.err = "BLAST chunk row capacity"; return false; }
  return true;
}

// Bit i set where block[i] is '\t' (low word) or '\n' (high word), 64 bytes at a time.
inline void sep_masks(const char* blk, uint64_t& tabs, uint64_t& nls) {
  const __m128i t = _mm_set1_epi8('\t'), n = _mm_set1_epi8('\n');
  tabs = nls = 0;
  for (int k = 0; k < 4; ++k) {
    const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(blk + 16 * k));
    tabs |= (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(x, t)) << (16 * k);
    nls |= (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(x, n)) << (16 * k);
  }
}

// The chunk's rows: tab and newline positions from 64-byte SSE2 masks (one pass over the
// bytes), the 15 fields of each row handed to parse_blast_row.  Same acceptance as
// split_tabs + line_end: exactly 14 tabs, no field starting with '"', a "\r\n" line end
// ending the text before the '\r', no empty line.
void parse_blast_chunk(Chunk& ck) {
  if (!all_plain(ck.b, ck.e)) { ck.err = "BLAST file has a lone CR, NUL or non-ASCII bytes"; return; }
  ck.rows.reserve((size_t)((ck.e - ck.b) / 30) + 2);   // (a row is >= 30 bytes)
  ck.ann.reserve((size_t)((ck.e - ck.b) / 2) + 2);     // (an annotation is >= 2 bytes: "|=", utils.py:239-241)
  sv f[15];
  int nf = 0;                                       // fields closed in the current row
  const char* fs = ck.b;                            // start of the current field
  auto bad_fields = [&]() { ck.err = "BLAST row without exactly 15 plain tab-separated fields"; };
  auto end_row = [&](const char* le) -> bool {      // le: the '\n' (or the chunk's end)
    const char* te = (le > fs && le[-1] == '\r') ? le - 1 : le;
    if (nf == 0 && te == fs) { ck.err = "empty BLAST line"; return false; }
    if (nf != 14 || (te > fs && *fs == '"')) { bad_fields(); return false; }
    f[14] = sv(fs, (size_t)(te - fs));
    if (!parse_blast_row(f, ck)) return false;
    nf = 0;
    fs = le + 1;
    return true;
  };
  const size_t n = (size_t)(ck.e - ck.b);
  char tail[64];
  for (size_t o = 0; o < n; o += 64) {
    const char* blk = ck.b + o;
    if (n - o < 64) {                                // the last partial block, padded
      memset(tail, ' ', 64);
      memcpy(tail, blk, n - o);
      blk = tail;
    }
    uint64_t tabs, nls;
    sep_masks(blk, tabs, nls);
    for (uint64_t m = tabs | nls; m; m &= m - 1) {
      const int i = __builtin_ctzll(m);
      const char* q = ck.b + o + i;
      if ((nls >> i) & 1ull) {
        if (!end_row(q)) return;
      } else {
        if (nf == 14 || *fs == '"') { bad_fields(); return; }
        f[nf++] = sv(fs, (size_t)(q - fs));
        fs = q + 1;
      }
    }
  }
  if (fs < ck.e || nf > 0) end_row(ck.e);            // a last line without '\n'
}

}  // namespace

// A plain array whose elements are left uninitialised on allocation: the parallel gather
// writes every element, so its pages are first touched by the threads that fill them
// (std::vector::resize would zero the whole array on the calling thread first).
struct wf_ingest {
  std::string err;
  bool ready = false;
  // contigs
  std::string contig_blob;
  std::vector<int64_t> contig_off, contig_length;
  // hits
  std::vector<int64_t> hit_off;
  PodArray<int64_t> hit_row;
  PodArray<int32_t> hit_group;          // run of its contig per hit (allocated only when a contig has several)
  PodArray<int32_t> hit_qlo, hit_qhi, hit_taxon, hit_value;
  PodArray<int8_t> hit_strand;
  PodArray<double> hit_score, hit_scov;
  PodArray<uint32_t> hit_sysmask;
  std::string taxa_blob, system_blob, value_blob;
  std::vector<int64_t> taxa_off, system_off, value_off;
  std::vector<int32_t> value_system;
  int32_t n_taxa = 0, n_systems = 0;
  int64_t n_values = 0;
  // loci
  std::vector<int64_t> loc_off, loc_strand_off;
  std::vector<int32_t> loc_start, loc_end;
  std::vector<int8_t> loc_strand;
  std::string loc_strand_blob;
  std::string loci_blob;                 // per contig: its LOCI field ("start:end:strand|...")
  std::vector<int64_t> loci_off;
  // warnings
  std::string warn_gff_blob, warn_blast_blob;
  std::vector<int64_t> warn_gff_off, warn_blast_off;
};

namespace {

void push_str(std::string& blob, std::vector<int64_t>& off, sv s) {
  if (off.empty()) off.push_back(0);
  blob.append(s.data(), s.size());
  off.push_back((int64_t)blob.size());
}

template <class F>
void parallel_for(int threads, int64_t n, F f) {
  if (threads <= 1 || n < 2) {
    for (int64_t i = 0; i < n; ++i) f(i, 0);
    return;
  }
  std::vector<std::thread> ts;
  std::atomic<int64_t> next{0};
  for (int t = 0; t < threads; ++t)
    ts.emplace_back([&, t]() {
      for (;;) {
        const int64_t i = next.fetch_add(1);
        if (i >= n) break;
        f(i, t);
      }
    });
  for (auto& th : ts) th.join();
}

// Cut [p, p + n) into `parts` pieces that start at line starts.
std::vector<std::pair<const char*, const char*>> line_chunks(const char* p, size_t n, int parts) {
  std::vector<std::pair<const char*, const char*>> out;
  const char* end = p + n;
  const char* s = p;
  for (int t = 0; t < parts; ++t) {
    const char* e = t == parts - 1 ? end : p + (n / parts) * (t + 1);
    if (e < s) e = s;
    if (e < end) {
      const char* nl = static_cast<const char*>(memchr(e, '\n', (size_t)(end - e)));
      e = nl ? nl + 1 : end;
    }
    out.emplace_back(s, e);
    s = e;
  }
  return out;
}

int chunk_count(int threads, size_t bytes) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(threads, (int64_t)(bytes / (1 << 20)) + 1));
}

// One piece of the FASTA file: the sequence length before its first header (`lead`), then
// each header's name with the length of the lines after it within the piece.
struct FaChunk {
  const char* b;
  const char* e;
  int64_t lead = 0;
  std::vector<std::pair<sv, int64_t>> heads;
  std::string err;
};

void scan_fasta_chunk(FaChunk& ck) {
  if (!all_plain(ck.b, ck.e)) { ck.err = "FASTA has a lone CR, NUL or non-ASCII bytes"; return; }
  const char* p = ck.b;
  int64_t acc = 0;                  // length since the last header (or the piece's start)
  bool in_head = false;
  while (p < ck.e) {
    const char* e;
    const char* le = line_end(p, ck.e, &e);
    const char* b = p;
    while (b < e && py_space((unsigned char)*b)) ++b;
    while (e > b && py_space((unsigned char)e[-1])) --e;
    if (b == e) { ck.err = "blank FASTA line"; return; }
    if (*b == '>') {
      const char* h = b + 1;
      while (h < e && py_space((unsigned char)*h)) ++h;
      const char* he = h;
      while (he < e && !py_space((unsigned char)*he)) ++he;
      if (he == h) { ck.err = "empty FASTA header"; return; }
      if (in_head) ck.heads.back().second = acc; else ck.lead = acc;
      ck.heads.emplace_back(sv(h, (size_t)(he - h)), 0);
      in_head = true;
      acc = 0;
    } else {
      acc += (int64_t)(e - b);
    }
    p = le < ck.e ? le + 1 : ck.e;
  }
  if (in_head) ck.heads.back().second = acc; else ck.lead = acc;
}

// read_contig_lengths (utils.py:109-120): OrderedDict semantics -- a repeated header
// resets its count but keeps its first position.  The pieces are scanned in parallel and
// applied in file order.
bool parse_fasta(const Mapped& m, wf_ingest& I, std::unordered_map<sv, int32_t>& index,
                 std::vector<sv>& names, int threads) {
  const auto parts = line_chunks(m.p, m.n, chunk_count(threads, m.n));
  std::vector<FaChunk> ck(parts.size());
  for (size_t t = 0; t < parts.size(); ++t) { ck[t].b = parts[t].first; ck[t].e = parts[t].second; }
  parallel_for(threads, (int64_t)ck.size(), [&](int64_t t, int) { scan_fasta_chunk(ck[t]); });
  int32_t cur = -1;
  for (const FaChunk& c : ck) {
    if (!c.err.empty()) { I.err = c.err; return false; }
    if (c.lead > 0) {
      if (cur < 0) { I.err = "sequence before the first FASTA header"; return false; }
      I.contig_length[cur] += c.lead;
    }
    for (const auto& h : c.heads) {
      auto it = index.find(h.first);
      if (it == index.end()) {
        cur = (int32_t)names.size();
        index.emplace(h.first, cur);
        names.push_back(h.first);
        I.contig_length.push_back(0);
      } else {
        cur = it->second;
        I.contig_length[cur] = 0;
      }
      I.contig_length[cur] += h.second;
    }
  }
  I.contig_off.assign(1, 0);
  for (const sv& n : names) push_str(I.contig_blob, I.contig_off, n);
  return true;
}

// iter_contig_loci + Locus (utils.py:300-355) and the length filter of
// orgscorer.py:348-357, grouped by consecutive seqname.
bool parse_gff(const Mapped& m, wf_ingest& I, const std::unordered_map<sv, int32_t>& index,
               int32_t N, double min_len) {
  if (!all_plain(m.p, m.p + m.n)) { I.err = "GFF has a lone CR, NUL or non-ASCII bytes"; return false; }
  struct Loc { int64_t s, e; sv strand; };
  std::vector<std::vector<Loc>> per((size_t)N);
  std::vector<char> seen((size_t)N, 0);
  I.warn_gff_off.assign(1, 0);
  const char* p = m.p;
  const char* end = m.p + m.n;
  sv cur;
  bool have = false;
  int32_t cur_c = -1;
  auto start_group = [&](sv name) -> bool {
    have = true;
    cur = name;
    auto it = index.find(name);
    cur_c = it == index.end() ? -1 : it->second;
    if (cur_c < 0) {
      push_str(I.warn_gff_blob, I.warn_gff_off, name);
    } else {
      if (seen[cur_c]) { I.err = "GFF loci of a contig are not contiguous"; return false; }
      seen[cur_c] = 1;
    }
    return true;
  };
  while (p < end) {
    const char* te;
    const char* le = line_end(p, end, &te);
    if (te == p || *p == '\t') { I.err = "empty GFF row or seqname"; return false; }
    if (*p != '#') {
      sv f[9];
      if (!split_tabs(p, te, f)) { I.err = "GFF row without exactly 9 plain tab-separated fields"; return false; }
      int64_t s, e;
      double sc;
      if (!parse_int(f[3], s) || !parse_int(f[4], e) || (f[5] != "." && !parse_float(f[5], sc))) {
        I.err = "GFF numeric field outside the plain spelling";
        return false;
      }
      if (!have || f[0] != cur)
        if (!start_group(f[0])) return false;
      if (cur_c >= 0) {
        const int64_t len = (e > s ? e - s : s - e) + 1;
        if ((double)len >= min_len) per[cur_c].push_back(Loc{s, e, f[6]});
      }
    }
    p = le < end ? le + 1 : end;
  }
  I.loc_off.assign((size_t)N + 1, 0);
  for (int32_t c = 0; c < N; ++c) I.loc_off[c + 1] = I.loc_off[c] + (int64_t)per[c].size();
  const int64_t L = I.loc_off[N];
  I.loc_start.resize((size_t)L);
  I.loc_end.resize((size_t)L);
  I.loc_strand.resize((size_t)L);
  I.loc_strand_off.assign(1, 0);
  int64_t k = 0;
  for (int32_t c = 0; c < N; ++c) {
    for (const Loc& l : per[c]) {
      if (l.s < INT32_MIN || l.s > INT32_MAX || l.e < INT32_MIN || l.e > INT32_MAX) {
        I.err = "gff start/end outside int32";
        return false;
      }
      I.loc_start[k] = (int32_t)l.s;
      I.loc_end[k] = (int32_t)l.e;
      I.loc_strand[k] = l.strand == "+" ? 0 : (l.strand == "-" ? 1 : 2);
      push_str(I.loc_strand_blob, I.loc_strand_off, l.strand);
      ++k;
    }
  }
  // each contig's LOCI field (orgscorer.py:795-800: Locus.code = "start:end:strand",
  // utils.py:312, the ints in Python's decimal spelling), joined by '|'
  I.loci_off.assign((size_t)N + 1, 0);
  I.loci_blob.reserve((size_t)L * 20);
  char buf[16];                          // an int32 is at most 11 characters
  for (int32_t c = 0; c < N; ++c) {
    for (int64_t j = I.loc_off[c]; j < I.loc_off[c + 1]; ++j) {
      if (j > I.loc_off[c]) I.loci_blob.push_back('|');
      I.loci_blob.append(buf, (size_t)(std::to_chars(buf, buf + sizeof buf, I.loc_start[j]).ptr - buf));
      I.loci_blob.push_back(':');
      I.loci_blob.append(buf, (size_t)(std::to_chars(buf, buf + sizeof buf, I.loc_end[j]).ptr - buf));
      I.loci_blob.push_back(':');
      const int64_t so = I.loc_strand_off[j];
      I.loci_blob.append(I.loc_strand_blob, (size_t)so, (size_t)(I.loc_strand_off[j + 1] - so));
    }
    I.loci_off[c + 1] = (int64_t)I.loci_blob.size();
  }
  return true;
}

// `side` (the GFF reader, which needs the FASTA's index) runs on the calling thread while
// the chunk threads parse BLAST rows; grouping starts once both are done.
template <class Side>
bool parse_blast(const Mapped& m, wf_ingest& I, const std::unordered_map<sv, int32_t>& index,
                 const int32_t& N, int threads, Side side) {
  const auto parts = line_chunks(m.p, m.n, chunk_count(threads, m.n));
  const int T = (int)parts.size();
  std::vector<Chunk> ck((size_t)T);
  for (int t = 0; t < T; ++t) { ck[t].b = parts[t].first; ck[t].e = parts[t].second; }
  bool side_ok = true;
  {
    std::vector<std::thread> ts;
    for (int t = 0; t < T; ++t) ts.emplace_back([&ck, t]() { parse_blast_chunk(ck[t]); });
    side_ok = side();
    for (auto& th : ts) th.join();
  }
  if (!side_ok) return false;
  for (auto& c : ck)
    if (!c.err.empty()) { I.err = c.err; return false; }

  // groups of consecutive qseqid (utils.py:262-266) -> FASTA contigs: the chunks' runs in
  // file order, a run continuing the previous chunk's last qseqid joining its group
  // rows [r0, r1) of a chunk; run: the contig's run number (a blastout not grouped by contig
  // keeps every run, in file order -- the caller scores it run by run, regroup.py)
  struct Piece { int32_t contig; int32_t chunk; int64_t r0, r1; int32_t run; };
  std::vector<Piece> runs;
  std::vector<int32_t> nrun((size_t)N, 0);
  bool regrouped = false;
  I.warn_blast_off.assign(1, 0);
  std::vector<int64_t> chunk_base((size_t)T + 1, 0);
  sv prev;
  bool have = false;
  for (int t = 0; t < T; ++t) {
    chunk_base[t + 1] = chunk_base[t] + (int64_t)ck[t].rows.size();
    for (const QRun& r : ck[t].runs) {
      if (have && r.q == prev) {                     // (only a chunk's first run can continue)
        runs.push_back(Piece{runs.back().contig, t, r.r0, r.r1, runs.back().run});
        continue;
      }
      have = true;
      prev = r.q;
      auto it = index.find(r.q);
      const int32_t c = it == index.end() ? -1 : it->second;
      int32_t run = 0;
      if (c < 0) {
        push_str(I.warn_blast_blob, I.warn_blast_off, r.q);
      } else {
        run = nrun[c]++;
        regrouped |= run > 0;
      }
      runs.push_back(Piece{c, t, r.r0, r.r1, run});
    }
  }
  std::vector<int64_t> counts((size_t)N, 0);
  for (const Piece& g : runs)
    if (g.contig >= 0) counts[g.contig] += g.r1 - g.r0;
  I.hit_off.assign((size_t)N + 1, 0);
  for (int32_t c = 0; c < N; ++c) I.hit_off[c + 1] = I.hit_off[c] + counts[c];
  const int64_t H = I.hit_off[N];
  // output position of each kept run
  std::vector<int64_t> run_dst(runs.size(), -1);
  {
    std::vector<int64_t> fill(I.hit_off.begin(), I.hit_off.end() - 1);
    for (size_t k = 0; k < runs.size(); ++k) {
      const Piece& g = runs[k];
      if (g.contig < 0) continue;
      run_dst[k] = fill[g.contig];
      fill[g.contig] += g.r1 - g.r0;
    }
  }
  // taxa / systems used by kept rows (the reference only sees the hits of known contigs:
  // orgscorer.py:944-946), per chunk in parallel; a kept row that failed its derivation or
  // its sseqid sends the file to the Python reader
  std::vector<std::vector<char>> tax_used(T), sys_used(T);
  std::vector<int> bad((size_t)T, 0);
  {
    std::vector<std::vector<int64_t>> chunk_runs(T);
    for (size_t k = 0; k < runs.size(); ++k)
      if (runs[k].contig >= 0) chunk_runs[runs[k].chunk].push_back((int64_t)k);
    parallel_for(threads, T, [&](int64_t t, int) {
      const Chunk& c = ck[t];
      tax_used[t].assign(c.taxa.names.size(), 0);
      sys_used[t].assign(c.systems.names.size(), 0);
      for (int64_t k : chunk_runs[t])
        for (int64_t i = runs[k].r0; i < runs[k].r1; ++i) {
          const Row& r = c.rows[i];
          if (r.taxon < 0) { bad[t] = 4; return; }
          if (r.bad) { bad[t] = r.bad; return; }
          tax_used[t][r.taxon] = 1;
          for (int32_t a = 0; a < r.ann_n; ++a) sys_used[t][c.ann[r.ann_off + a].first] = 1;
        }
    });
  }
  for (int t = 0; t < T; ++t)
    if (bad[t]) {
      I.err = bad[t] == 4 ? "bad subject id header or annotation in a kept BLAST row"
              : bad[t] == 1 ? "slen or qlen is 0 in a BLAST row"
              : bad[t] == 2 ? "scov_modified denominator is 0" : "qstart/qend outside int32";
      return false;
    }
  std::vector<std::vector<int32_t>> tax_g(T), sys_g(T);
  std::vector<int32_t> val_base((size_t)T + 1, 0);
  {
    std::unordered_map<sv, int32_t> tg;
    I.taxa_off.assign(1, 0);
    std::map<std::string, int32_t> sg;     // sorted systems (orgscorer: sorted(set(...)))
    for (int t = 0; t < T; ++t) {
      tax_g[t].assign(ck[t].taxa.names.size(), -1);
      for (size_t j = 0; j < ck[t].taxa.names.size(); ++j) {
        if (!tax_used[t][j]) continue;
        const sv n = ck[t].taxa.names[j];
        auto it = tg.find(n);
        if (it == tg.end()) {
          it = tg.emplace(n, (int32_t)tg.size()).first;
          push_str(I.taxa_blob, I.taxa_off, n);
        }
        tax_g[t][j] = it->second;
      }
      for (size_t j = 0; j < ck[t].systems.names.size(); ++j)
        if (sys_used[t][j]) sg.emplace(std::string(ck[t].systems.names[j]), 0);
    }
    I.n_taxa = (int32_t)tg.size();
    int32_t b = 0;
    I.system_off.assign(1, 0);
    for (auto& kv : sg) {
      kv.second = b++;
      push_str(I.system_blob, I.system_off, kv.first);
    }
    I.n_systems = b;
    if (I.n_systems > 32) { I.err = "more than 32 annotation systems"; return false; }
    // annotation values: thread tables concatenated (ids = thread base + local id); a text
    // may repeat across threads, which only the rendering (by id) ever sees
    I.value_off.assign(1, 0);
    for (int t = 0; t < T; ++t) {
      sys_g[t].assign(ck[t].systems.names.size(), -1);
      for (size_t j = 0; j < ck[t].systems.names.size(); ++j)
        if (sys_used[t][j]) sys_g[t][j] = sg[std::string(ck[t].systems.names[j])];
      val_base[t + 1] = val_base[t] + (int32_t)ck[t].value_sys.size();
      for (size_t j = 0; j < ck[t].value_sys.size(); ++j) {
        I.value_system.push_back(sys_g[t][ck[t].value_sys[j]]);
        push_str(I.value_blob, I.value_off, ck[t].values.texts[j]);
      }
    }
    I.n_values = (int64_t)I.value_system.size();
  }
  // gather kept rows into FASTA contig order
  I.hit_qlo.alloc((size_t)H); I.hit_qhi.alloc((size_t)H); I.hit_taxon.alloc((size_t)H);
  I.hit_strand.alloc((size_t)H); I.hit_score.alloc((size_t)H); I.hit_scov.alloc((size_t)H);
  I.hit_sysmask.alloc((size_t)H); I.hit_row.alloc((size_t)H);
  if (regrouped) I.hit_group.alloc((size_t)H);
  const int S = std::max(1, (int)I.n_systems);
  I.hit_value.alloc((size_t)H * S);
  parallel_for(threads, (int64_t)runs.size(), [&](int64_t k, int) {
    const Piece& g = runs[k];
    if (g.contig < 0) return;
    const Chunk& c = ck[g.chunk];
    const int32_t* tmap = tax_g[g.chunk].data();
    const int32_t* smap = sys_g[g.chunk].data();
    const int32_t vb = val_base[g.chunk];
    int64_t o = run_dst[k];
    for (int64_t i = g.r0; i < g.r1; ++i, ++o) {
      const Row& r = c.rows[i];
      I.hit_qlo[o] = r.qlo;
      I.hit_qhi[o] = r.qhi;
      I.hit_taxon[o] = tmap[r.taxon];
      I.hit_strand[o] = (int8_t)r.minus;
      I.hit_scov[o] = r.scov;
      I.hit_score[o] = r.score;
      I.hit_row[o] = chunk_base[g.chunk] + i;
      if (regrouped) I.hit_group[o] = g.run;
      int32_t* hv = &I.hit_value[(size_t)o * S];
      for (int b = 0; b < S; ++b) hv[b] = -1;
      uint32_t mask = 0;
      for (int32_t a = 0; a < r.ann_n; ++a) {             // later duplicates win (dict)
        const auto& av = c.ann[r.ann_off + a];
        const int32_t b = smap[av.first];
        mask |= 1u << b;
        hv[b] = vb + av.second;
      }
      I.hit_sysmask[o] = mask;
    }
  });
  return true;
}

}  // namespace

extern "C" {

int wf_ingest_abi_version(void) { return WF_INGEST_ABI_VERSION; }

wf_ingest* wf_ingest_new(void) { return new (std::nothrow) wf_ingest(); }

void wf_ingest_free(wf_ingest* ing) { delete ing; }

const char* wf_ingest_last_error(const wf_ingest* ing) { return ing ? ing->err.c_str() : "null ingest"; }

int wf_ingest_parse(wf_ingest* ing, const char* fasta_path, const char* blastout_path,
                    const char* gff_path, double min_gene_length, int threads) {
  if (!ing || !fasta_path || !blastout_path || !gff_path) return WF_INGEST_E_STATE;
  wf_ingest& I = *ing;
  I = wf_ingest();
  if (threads <= 0) threads = (int)std::max(1u, std::min(64u, std::thread::hardware_concurrency()));
  Mapped fa, bl, gf;
  if (!fa.open(fasta_path, &I.err) || !bl.open(blastout_path, &I.err) || !gf.open(gff_path, &I.err))
    return WF_INGEST_E_IO;
  std::unordered_map<sv, int32_t> index;
  std::vector<sv> names;
  try {
    int32_t N = 0;
    // the reference reads the GFF before the BLAST file (orgscorer.py:948-951); here the
    // FASTA pieces are scanned in parallel first, then the GFF reader runs while the BLAST
    // chunks are parsed
    if (!parse_fasta(fa, I, index, names, threads)) return WF_INGEST_FALLBACK;
    N = (int32_t)names.size();
    auto side = [&]() { return parse_gff(gf, I, index, N, min_gene_length); };
    if (!parse_blast(bl, I, index, N, threads, side)) return WF_INGEST_FALLBACK;
  } catch (const std::bad_alloc&) {
    I.err = "out of host memory while parsing";
    return WF_INGEST_FALLBACK;
  }
  I.ready = true;
  return WF_INGEST_OK;
}

int wf_ingest_get_view(const wf_ingest* ing, wf_ingest_view* v) {
  if (!ing || !v || !ing->ready) return WF_INGEST_E_STATE;
  const wf_ingest& I = *ing;
  *v = wf_ingest_view{};
  v->n_contigs = (int32_t)I.contig_length.size();
  v->n_taxa = I.n_taxa;
  v->n_systems = I.n_systems;
  v->n_warn_gff = (int32_t)I.warn_gff_off.size() - 1;
  v->n_warn_blast = (int32_t)I.warn_blast_off.size() - 1;
  v->n_hits = I.hit_off.empty() ? 0 : I.hit_off.back();
  v->n_loci = I.loc_off.empty() ? 0 : I.loc_off.back();
  v->n_values = I.n_values;
  v->contig_blob = I.contig_blob.data(); v->contig_off = I.contig_off.data();
  v->contig_length = I.contig_length.data();
  v->hit_off = I.hit_off.data(); v->hit_qlo = I.hit_qlo.data(); v->hit_qhi = I.hit_qhi.data();
  v->hit_taxon = I.hit_taxon.data(); v->hit_strand = I.hit_strand.data();
  v->hit_score = I.hit_score.data(); v->hit_scov = I.hit_scov.data();
  v->hit_sysmask = I.hit_sysmask.data(); v->hit_row = I.hit_row.data();
  v->hit_value = I.hit_value.data();
  v->hit_group = I.hit_group.data();
  v->taxa_blob = I.taxa_blob.data(); v->taxa_off = I.taxa_off.data();
  v->system_blob = I.system_blob.data(); v->system_off = I.system_off.data();
  v->value_blob = I.value_blob.data(); v->value_off = I.value_off.data();
  v->value_system = I.value_system.data();
  v->loc_off = I.loc_off.data(); v->loc_start = I.loc_start.data(); v->loc_end = I.loc_end.data();
  v->loc_strand = I.loc_strand.data();
  v->loc_strand_blob = I.loc_strand_blob.data(); v->loc_strand_off = I.loc_strand_off.data();
  v->warn_gff_blob = I.warn_gff_blob.data(); v->warn_gff_off = I.warn_gff_off.data();
  v->warn_blast_blob = I.warn_blast_blob.data(); v->warn_blast_off = I.warn_blast_off.data();
  v->loci_blob = I.loci_blob.data(); v->loci_off = I.loci_off.data();
  return WF_INGEST_OK;
}

}  // extern "C"
