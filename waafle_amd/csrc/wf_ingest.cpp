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
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

using sv = std::string_view;

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
  for (const char* q = b; q < e; ++q) {
    const unsigned char c = (unsigned char)*q;
    if (c >= 0x80 || c == 0) return false;
    if (c == '\r' && q + 1 < e && q[1] != '\n') return false;
  }
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

// [+-]?[0-9]+ into int64 (no overflow).
bool parse_int(sv f, int64_t& out) {
  size_t i = 0;
  bool neg = false;
  if (i < f.size() && (f[i] == '+' || f[i] == '-')) { neg = f[i] == '-'; ++i; }
  if (i == f.size()) return false;
  uint64_t v = 0;
  for (; i < f.size(); ++i) {
    const unsigned d = (unsigned)(f[i] - '0');
    if (d > 9) return false;
    if (v > (uint64_t)INT64_MAX / 10) return false;
    v = v * 10 + d;
    if (v > (uint64_t)INT64_MAX) return false;
  }
  out = neg ? -(int64_t)v : (int64_t)v;
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

struct Interner {
  std::unordered_map<sv, int32_t> idx;
  std::vector<sv> names;
  int32_t get(sv s) {
    auto it = idx.find(s);
    if (it != idx.end()) return it->second;
    const int32_t i = (int32_t)names.size();
    idx.emplace(s, i);
    names.push_back(s);
    return i;
  }
};

// (system id, value text): annotation values are interned per system without copying text.
struct SysVal {
  int32_t sys;
  sv val;
  bool operator==(const SysVal& o) const { return sys == o.sys && val == o.val; }
};
struct SysValHash {
  size_t operator()(const SysVal& k) const {
    return std::hash<sv>()(k.val) ^ ((size_t)(uint32_t)k.sys * 0x9E3779B97F4A7C15ull);
  }
};

struct Row {
  sv q;                           // qseqid
  int64_t qlen, slen, qstart, qend, sstart, send;
  double pident;
  int32_t taxon;                  // thread-local taxon id (-1: bad sseqid)
  int32_t ann_off, ann_n;         // thread-local annotation pairs
  bool minus;
};

struct Chunk {
  const char* b;
  const char* e;
  std::vector<Row> rows;
  std::vector<std::pair<int32_t, int32_t>> ann;   // (local system, local value)
  Interner taxa, systems;
  std::unordered_map<SysVal, int32_t, SysValHash> values;   // (local system, text) -> id
  std::vector<int32_t> value_sys;                 // local system of each local value
  std::vector<sv> value_text;
  std::string err;                                // non-empty: fallback
};

// One BLAST row (utils.py:207-241).  Numeric columns are validated for every row, as the
// reference converts every field of every row; sseqid problems are recorded and only
// matter for rows of known contigs.
bool parse_blast_row(const char* b, const char* e, Chunk& ck) {
  sv f[15];
  if (!split_tabs(b, e, f)) { ck.err = "BLAST row without exactly 15 plain tab-separated fields"; return false; }
  Row r;
  int64_t dummy;
  double dd;
  if (!parse_int(f[2], r.qlen) || !parse_int(f[3], r.slen) || !parse_int(f[4], dummy) ||
      !parse_int(f[5], r.qstart) || !parse_int(f[6], r.qend) || !parse_int(f[7], r.sstart) ||
      !parse_int(f[8], r.send) || !parse_int(f[10], dummy) || !parse_int(f[11], dummy)) {
    ck.err = "BLAST integer field outside the plain spelling";
    return false;
  }
  if (!parse_float(f[9], r.pident) || !parse_float(f[12], dd) || !parse_float(f[13], dd)) {
    ck.err = "BLAST float field outside the plain spelling";
    return false;
  }
  r.q = f[0];
  r.minus = f[14] == "minus";
  // sseqid: gene | taxon | system=value ... (utils.py:231-241)
  const sv sid = f[1];
  r.taxon = -1;
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
      if (eq == sv::npos || item.find('=', eq + 1) != sv::npos) { ok = false; break; }
      const sv sys = item.substr(0, eq), val = item.substr(eq + 1);
      const int32_t s = ck.systems.get(sys);
      auto it = ck.values.find(SysVal{s, val});
      int32_t v;
      if (it != ck.values.end()) {
        v = it->second;
      } else {
        v = (int32_t)ck.value_sys.size();
        ck.values.emplace(SysVal{s, val}, v);
        ck.value_sys.push_back(s);
        ck.value_text.push_back(val);
      }
      ck.ann.emplace_back(s, v);
      ++r.ann_n;
      p2 = p3;
    }
    if (ok) r.taxon = ck.taxa.get(taxon);
  }
  ck.rows.push_back(r);
  return true;
}

void parse_blast_chunk(Chunk& ck) {
  if (!all_plain(ck.b, ck.e)) { ck.err = "BLAST file has a lone CR, NUL or non-ASCII bytes"; return; }
  const char* p = ck.b;
  while (p < ck.e) {
    const char* te;
    const char* le = line_end(p, ck.e, &te);
    if (te == p) { ck.err = "empty BLAST line"; return; }
    if (!parse_blast_row(p, te, ck)) return;
    p = le < ck.e ? le + 1 : ck.e;
  }
}

}  // namespace

struct wf_ingest {
  std::string err;
  bool ready = false;
  // contigs
  std::string contig_blob;
  std::vector<int64_t> contig_off, contig_length;
  // hits
  std::vector<int64_t> hit_off, hit_row;
  std::vector<int32_t> hit_qlo, hit_qhi, hit_taxon, hit_value;
  std::vector<int8_t> hit_strand;
  std::vector<double> hit_score, hit_scov;
  std::vector<uint32_t> hit_sysmask;
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

// read_contig_lengths (utils.py:109-120): OrderedDict semantics -- a repeated header
// resets its count but keeps its first position.
bool parse_fasta(const Mapped& m, wf_ingest& I, std::unordered_map<sv, int32_t>& index,
                 std::vector<sv>& names) {
  if (!all_plain(m.p, m.p + m.n)) { I.err = "FASTA has a lone CR, NUL or non-ASCII bytes"; return false; }
  const char* p = m.p;
  const char* end = m.p + m.n;
  int32_t cur = -1;
  while (p < end) {
    const char* e;
    const char* le = line_end(p, end, &e);
    const char* b = p;
    while (b < e && py_space((unsigned char)*b)) ++b;
    while (e > b && py_space((unsigned char)e[-1])) --e;
    if (b == e) { I.err = "blank FASTA line"; return false; }
    if (*b == '>') {
      const char* h = b + 1;
      while (h < e && py_space((unsigned char)*h)) ++h;
      const char* he = h;
      while (he < e && !py_space((unsigned char)*he)) ++he;
      if (he == h) { I.err = "empty FASTA header"; return false; }
      const sv name(h, (size_t)(he - h));
      auto it = index.find(name);
      if (it == index.end()) {
        cur = (int32_t)names.size();
        index.emplace(name, cur);
        names.push_back(name);
        I.contig_length.push_back(0);
      } else {
        cur = it->second;
        I.contig_length[cur] = 0;
      }
    } else {
      if (cur < 0) { I.err = "sequence before the first FASTA header"; return false; }
      I.contig_length[cur] += (int64_t)(e - b);
    }
    p = le < end ? le + 1 : end;
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
  return true;
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

// `side` (the FASTA and GFF readers, which build `index` and N) runs on the calling thread
// while the chunk threads parse BLAST rows; grouping starts once both are done.
template <class Side>
bool parse_blast(const Mapped& m, wf_ingest& I, const std::unordered_map<sv, int32_t>& index,
                 const int32_t& N, int threads, Side side) {
  const char* end = m.p + m.n;
  // chunks at line boundaries
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(threads, (int64_t)(m.n / (1 << 20)) + 1));
  std::vector<Chunk> ck((size_t)T);
  const char* s = m.p;
  for (int t = 0; t < T; ++t) {
    const char* e = t == T - 1 ? end : m.p + (m.n / T) * (t + 1);
    if (e < s) e = s;
    if (e < end) {
      const char* nl = static_cast<const char*>(memchr(e, '\n', (size_t)(end - e)));
      e = nl ? nl + 1 : end;
    }
    ck[t].b = s;
    ck[t].e = e;
    s = e;
  }
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

  // groups of consecutive qseqid (utils.py:262-266) -> FASTA contigs
  struct Group { int32_t contig; int32_t chunk; int64_t r0, r1; };   // rows [r0, r1) of a chunk run
  std::vector<Group> runs;          // a group can span chunks: one run per chunk piece
  std::vector<int32_t> run_group;   // group index of each run
  std::vector<int32_t> group_contig;
  std::vector<char> seen((size_t)N, 0);
  I.warn_blast_off.assign(1, 0);
  sv prev;
  bool have = false;
  int64_t row_base = 0;
  std::vector<int64_t> chunk_base((size_t)T);
  for (int t = 0; t < T; ++t) {
    chunk_base[t] = row_base;
    const auto& rows = ck[t].rows;
    const int64_t n = (int64_t)rows.size();
    for (int64_t i = 0; i < n; ++i) {
      const sv q = rows[i].q;
      if (!have || q != prev) {
        have = true;
        prev = q;
        auto it = index.find(q);
        const int32_t c = it == index.end() ? -1 : it->second;
        if (c < 0) {
          push_str(I.warn_blast_blob, I.warn_blast_off, q);
        } else {
          if (seen[c]) { I.err = "BLAST hits of a contig are not contiguous"; return false; }
          seen[c] = 1;
        }
        group_contig.push_back(c);
        runs.push_back(Group{c, t, i, i});
        run_group.push_back((int32_t)group_contig.size() - 1);
      } else if (runs.back().chunk != t) {
        runs.push_back(Group{runs.back().contig, t, i, i});
        run_group.push_back(run_group.back());
      }
      runs.back().r1 = i + 1;
    }
    row_base += n;
  }
  std::vector<int64_t> counts((size_t)N, 0);
  for (const Group& g : runs)
    if (g.contig >= 0) counts[g.contig] += g.r1 - g.r0;
  I.hit_off.assign((size_t)N + 1, 0);
  for (int32_t c = 0; c < N; ++c) I.hit_off[c + 1] = I.hit_off[c] + counts[c];
  const int64_t H = I.hit_off[N];
  // output position of each kept run
  std::vector<int64_t> run_dst(runs.size(), -1);
  {
    std::vector<int64_t> fill(I.hit_off.begin(), I.hit_off.end() - 1);
    for (size_t k = 0; k < runs.size(); ++k) {
      const Group& g = runs[k];
      if (g.contig < 0) continue;
      run_dst[k] = fill[g.contig];
      fill[g.contig] += g.r1 - g.r0;
    }
  }
  // taxa / systems / values used by kept rows -> global ids (the reference only sees the
  // hits of known contigs: orgscorer.py:944-946)
  std::vector<std::vector<char>> tax_used(T), sys_used(T);
  for (int t = 0; t < T; ++t) {
    tax_used[t].assign(ck[t].taxa.names.size(), 0);
    sys_used[t].assign(ck[t].systems.names.size(), 0);
  }
  for (size_t k = 0; k < runs.size(); ++k) {
    const Group& g = runs[k];
    if (g.contig < 0) continue;
    const Chunk& c = ck[g.chunk];
    for (int64_t i = g.r0; i < g.r1; ++i) {
      const Row& r = c.rows[i];
      if (r.taxon < 0) { I.err = "bad subject id header or annotation in a kept BLAST row"; return false; }
      tax_used[g.chunk][r.taxon] = 1;
      for (int32_t a = 0; a < r.ann_n; ++a) sys_used[g.chunk][c.ann[r.ann_off + a].first] = 1;
    }
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
        push_str(I.value_blob, I.value_off, ck[t].value_text[j]);
      }
    }
    I.n_values = (int64_t)I.value_system.size();
  }
  // gather kept rows into FASTA contig order and derive the hit values
  I.hit_qlo.resize((size_t)H); I.hit_qhi.resize((size_t)H); I.hit_taxon.resize((size_t)H);
  I.hit_strand.resize((size_t)H); I.hit_score.resize((size_t)H); I.hit_scov.resize((size_t)H);
  I.hit_sysmask.resize((size_t)H); I.hit_row.resize((size_t)H);
  const int S = std::max(1, (int)I.n_systems);
  I.hit_value.assign((size_t)H * S, -1);
  std::atomic<int> why{0};
  parallel_for(threads, (int64_t)runs.size(), [&](int64_t k, int) {
    const Group& g = runs[k];
    if (g.contig < 0) return;
    const Chunk& c = ck[g.chunk];
    int64_t o = run_dst[k];
    for (int64_t i = g.r0; i < g.r1; ++i, ++o) {
      const Row& r = c.rows[i];
      // utils.py:216-229, evaluated as the reference does (int64, then float64)
      if (r.slen == 0 || r.qlen == 0) { why = 1; return; }
      const int64_t s0 = r.minus ? r.slen - r.sstart + 1 : r.sstart;
      const int64_t s1 = r.minus ? r.slen - r.send + 1 : r.send;
      const int64_t ltrim = std::max<int64_t>(0, s0 - r.qstart);
      const int64_t rtrim = std::max<int64_t>(0, r.slen - s0 - r.qlen + r.qstart);
      const int64_t den = r.slen - ltrim - rtrim;
      if (den == 0) { why = 2; return; }
      const double scov = (double)(s1 - s0 + 1) / (double)den;
      const double score = scov * r.pident / 100.0;
      if (r.qstart < INT32_MIN || r.qstart > INT32_MAX || r.qend < INT32_MIN || r.qend > INT32_MAX) {
        why = 3;
        return;
      }
      I.hit_qlo[o] = (int32_t)std::min(r.qstart, r.qend);
      I.hit_qhi[o] = (int32_t)std::max(r.qstart, r.qend);
      I.hit_taxon[o] = tax_g[g.chunk][r.taxon];
      I.hit_strand[o] = r.minus ? 1 : 0;
      I.hit_scov[o] = scov;
      I.hit_score[o] = score;
      I.hit_row[o] = chunk_base[g.chunk] + i;
      uint32_t mask = 0;
      for (int32_t a = 0; a < r.ann_n; ++a) {             // later duplicates win (dict)
        const int32_t b = sys_g[g.chunk][c.ann[r.ann_off + a].first];
        mask |= 1u << b;
        I.hit_value[(size_t)o * S + b] = val_base[g.chunk] + c.ann[r.ann_off + a].second;
      }
      I.hit_sysmask[o] = mask;
    }
  });
  if (why) {
    I.err = why == 1 ? "slen or qlen is 0 in a BLAST row"
                     : why == 2 ? "scov_modified denominator is 0" : "qstart/qend outside int32";
    return false;
  }
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
    // FASTA and GFF readers run while the BLAST chunks are parsed
    auto side = [&]() {
      if (!parse_fasta(fa, I, index, names)) return false;
      N = (int32_t)names.size();
      return parse_gff(gf, I, index, N, min_gene_length);
    };
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
  v->taxa_blob = I.taxa_blob.data(); v->taxa_off = I.taxa_off.data();
  v->system_blob = I.system_blob.data(); v->system_off = I.system_off.data();
  v->value_blob = I.value_blob.data(); v->value_off = I.value_off.data();
  v->value_system = I.value_system.data();
  v->loc_off = I.loc_off.data(); v->loc_start = I.loc_start.data(); v->loc_end = I.loc_end.data();
  v->loc_strand = I.loc_strand.data();
  v->loc_strand_blob = I.loc_strand_blob.data(); v->loc_strand_off = I.loc_strand_off.data();
  v->warn_gff_blob = I.warn_gff_blob.data(); v->warn_gff_off = I.warn_gff_off.data();
  v->warn_blast_blob = I.warn_blast_blob.data(); v->warn_blast_off = I.warn_blast_off.data();
  return WF_INGEST_OK;
}

}  // extern "C"
