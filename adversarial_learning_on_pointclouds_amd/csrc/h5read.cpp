// HDF5-free reader for the point-cloud datasets of the reference
// (dataset/modelNetData.py:43-47 and dataset/shapeNetData.py:176-181 read
// f['data'][:, 0:npts, :], f['label'][:] and f['pid'][:, 0:npts] through h5py;
// h5py is not part of this image).  Host code only: it parses the on-disk
// format directly from a read-only mapping of the file and converts the
// dataset to f32 or int64.
//
// Supported (what HDF5 1.8 - 1.12 writes for these files, including PointNet's
// gzip-chunked ModelNet40 / ShapeNet-part files):
//   superblock v0 / v1 (libver 'earliest': v1 object headers, symbol-table
//   groups: B-tree v1 + local heap + SNOD) and v2 / v3 (libver 'latest': v2
//   object headers, compact link messages);
//   datasets of fixed-point (1/2/4/8 B, signed or not) or IEEE float (4/8 B)
//   elements, either byte order;
//   layouts: compact, contiguous, chunked with a v1 B-tree index (layout v3),
//   or (layout v4) single-chunk, implicit and non-paged fixed-array indexes;
//   filters: deflate (zlib) and shuffle (fletcher32 checksums are skipped).
// Anything else (dense link storage, extensible-array / v2 B-tree chunk
// indexes, other filters, external storage) fails with a message naming it.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "pcadv.h"

namespace pcadv {
void set_error(const char* fmt, ...);
}

namespace {

struct H5Error {
  std::string msg;
};

[[noreturn]] void fail(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  throw H5Error{buf};
}

constexpr uint64_t UNDEF = ~0ull;

struct File {
  const uint8_t* p = nullptr;
  size_t n = 0;
  int fd = -1;
  int so = 8, sl = 8;  // sizes of offsets and lengths
  uint64_t base = 0;
  ~File() {
    if (p) munmap(const_cast<uint8_t*>(p), n);
    if (fd >= 0) close(fd);
  }
  void need(uint64_t off, uint64_t len) const {
    if (off > n || len > n - off) fail("truncated file: %llu + %llu > %zu", (unsigned long long)off,
                                       (unsigned long long)len, n);
  }
  uint64_t u(uint64_t off, int bytes) const {
    need(off, bytes);
    uint64_t v = 0;
    for (int i = bytes - 1; i >= 0; --i) v = (v << 8) | p[off + i];
    return v;
  }
  uint64_t addr(uint64_t off) const {
    const uint64_t v = u(off, so);
    if (so == 8 && v == UNDEF) return UNDEF;
    if (so == 4 && v == 0xffffffffull) return UNDEF;
    return v + base;
  }
  uint64_t len(uint64_t off) const { return u(off, sl); }
  bool sig(uint64_t off, const char* s) const {
    need(off, 4);
    return std::memcmp(p + off, s, 4) == 0;
  }
};

struct Msg {
  int type;
  uint64_t off, size;
};

// ---- object headers: the list of messages (continuations followed) --------
std::vector<Msg> object_messages(const File& f, uint64_t oh) {
  std::vector<Msg> out;
  if (f.sig(oh, "OHDR")) {  // version 2
    const int flags = (int)f.u(oh + 5, 1);
    uint64_t q = oh + 6;
    if (flags & 0x20) q += 16;
    if (flags & 0x10) q += 4;
    const int csz = 1 << (flags & 3);
    uint64_t chunk_len = f.u(q, csz);
    q += csz;
    const bool crt = flags & 0x04;
    std::vector<std::pair<uint64_t, uint64_t>> blocks{{q, chunk_len}};
    for (size_t b = 0; b < blocks.size(); ++b) {
      uint64_t m = blocks[b].first, end = blocks[b].first + blocks[b].second;
      while (m + 4 <= end) {
        const int type = (int)f.u(m, 1);
        const uint64_t size = f.u(m + 1, 2);
        const uint64_t data = m + 4 + (crt ? 2 : 0);
        if (data + size > end) break;
        if (type == 0x10) {  // continuation: "OCHK" + messages + checksum
          const uint64_t a = f.addr(data), l = f.len(data + f.so);
          if (!f.sig(a, "OCHK")) fail("bad v2 continuation block");
          blocks.push_back({a + 4, l - 8});
        } else if (type != 0) {
          out.push_back({type, data, size});
        }
        m = data + size;
      }
    }
    return out;
  }
  if (f.u(oh, 1) != 1) fail("unsupported object header version %d", (int)f.u(oh, 1));
  const uint64_t nmsg = f.u(oh + 2, 2);
  const uint64_t hsize = f.u(oh + 8, 4);
  std::vector<std::pair<uint64_t, uint64_t>> blocks{{oh + 16, hsize}};
  uint64_t seen = 0;
  for (size_t b = 0; b < blocks.size() && seen < nmsg; ++b) {
    uint64_t m = blocks[b].first, end = blocks[b].first + blocks[b].second;
    while (m + 8 <= end && seen < nmsg) {
      const int type = (int)f.u(m, 2);
      const uint64_t size = f.u(m + 2, 2);
      const uint64_t data = m + 8;
      ++seen;
      if (type == 0x10) blocks.push_back({f.addr(data), f.len(data + f.so)});
      else if (type != 0) out.push_back({type, data, size});
      m = data + size;
    }
  }
  return out;
}

const Msg* find(const std::vector<Msg>& ms, int type) {
  for (const Msg& m : ms)
    if (m.type == type) return &m;
  return nullptr;
}

// ---- groups ---------------------------------------------------------------
std::string heap_string(const File& f, uint64_t heap_data, uint64_t off) {
  f.need(heap_data + off, 1);
  const char* s = reinterpret_cast<const char*>(f.p + heap_data + off);
  return std::string(s, strnlen(s, f.n - (heap_data + off)));
}

// symbol-table group: walk the v1 B-tree (type 0) down to the SNOD leaves
uint64_t lookup_symtab(const File& f, uint64_t btree, uint64_t heap, const std::string& name) {
  if (!f.sig(heap, "HEAP")) fail("bad local heap signature");
  const uint64_t heap_data = f.addr(heap + 8 + 2 * f.sl);
  std::vector<uint64_t> stack{btree};
  while (!stack.empty()) {
    const uint64_t node = stack.back();
    stack.pop_back();
    if (f.sig(node, "TREE")) {
      const int type = (int)f.u(node + 4, 1), level = (int)f.u(node + 5, 1);
      const int used = (int)f.u(node + 6, 2);
      if (type != 0) fail("group B-tree of type %d", type);
      uint64_t q = node + 8 + 2 * f.so + f.sl;  // first child (after key 0)
      for (int i = 0; i < used; ++i) {
        stack.push_back(f.addr(q));
        q += f.so + f.sl;
      }
      (void)level;
    } else if (f.sig(node, "SNOD")) {
      const int nsym = (int)f.u(node + 6, 2);
      uint64_t e = node + 8;
      for (int i = 0; i < nsym; ++i) {
        if (heap_string(f, heap_data, f.len(e)) == name) return f.addr(e + f.so);
        e += 2 * f.so + 8 + 16;
      }
    } else {
      fail("bad group node signature");
    }
  }
  return UNDEF;
}

uint64_t lookup(const File& f, uint64_t group_oh, const std::string& name) {
  const std::vector<Msg> ms = object_messages(f, group_oh);
  if (const Msg* st = find(ms, 0x11)) return lookup_symtab(f, f.addr(st->off), f.addr(st->off + f.so), name);
  for (const Msg& m : ms) {
    if (m.type != 0x06) continue;  // link message
    const int flags = (int)f.u(m.off + 1, 1);
    uint64_t q = m.off + 2;
    int ltype = 0;
    if (flags & 0x08) ltype = (int)f.u(q++, 1);
    if (flags & 0x04) q += 8;
    if (flags & 0x10) q += 1;
    const int lsz = 1 << (flags & 3);
    const uint64_t nlen = f.u(q, lsz);
    q += lsz;
    f.need(q, nlen);
    const std::string nm(reinterpret_cast<const char*>(f.p + q), nlen);
    q += nlen;
    if (nm == name) {
      if (ltype != 0) fail("'%s' is not a hard link", name.c_str());
      return f.addr(q);
    }
  }
  if (find(ms, 0x02)) fail("dense link storage (fractal heap) is not supported");
  return UNDEF;
}

// ---- datasets -------------------------------------------------------------
struct Dataset {
  std::vector<uint64_t> dims;
  int klass = 0, esize = 0;  // 0 fixed-point, 1 float
  bool is_signed = false, big_endian = false;
  std::vector<int> filters;  // filter ids in pipeline (write) order
  std::vector<uint8_t> raw;  // all elements, native layout
};

uint64_t count(const std::vector<uint64_t>& d) {
  uint64_t n = 1;
  for (uint64_t v : d) n *= v;
  return n;
}

void parse_dataspace(const File& f, const Msg& m, Dataset& ds) {
  const int ver = (int)f.u(m.off, 1), rank = (int)f.u(m.off + 1, 1);
  uint64_t q = m.off + (ver == 1 ? 8 : 4);
  if (ver == 2 && f.u(m.off + 3, 1) == 2) fail("null dataspace");
  for (int i = 0; i < rank; ++i) ds.dims.push_back(f.len(q + (uint64_t)i * f.sl));
}

void parse_datatype(const File& f, const Msg& m, Dataset& ds) {
  const int cv = (int)f.u(m.off, 1), bits = (int)f.u(m.off + 1, 1);
  ds.klass = cv & 15;
  ds.esize = (int)f.u(m.off + 4, 4);
  ds.big_endian = bits & 1;
  if (ds.klass == 0) {
    ds.is_signed = bits & 8;
    if (ds.esize != 1 && ds.esize != 2 && ds.esize != 4 && ds.esize != 8) fail("integer size %d", ds.esize);
  } else if (ds.klass == 1) {
    if (ds.esize != 4 && ds.esize != 8) fail("float size %d", ds.esize);
    if (bits & 0x40) fail("VAX float order");
  } else {
    fail("datatype class %d is not numeric", ds.klass);
  }
}

void parse_filters(const File& f, const Msg& m, Dataset& ds) {
  const int ver = (int)f.u(m.off, 1), nf = (int)f.u(m.off + 1, 1);
  uint64_t q = m.off + (ver == 1 ? 8 : 2);
  for (int i = 0; i < nf; ++i) {
    const int id = (int)f.u(q, 2);
    uint64_t namelen = 0;
    if (ver == 1 || id >= 256) {
      namelen = f.u(q + 2, 2);
      q += 2;
    }
    const int ncd = (int)f.u(q + 4, 2);
    q += 6;
    if (ver == 1) namelen = (namelen + 7) & ~7ull;
    q += namelen + 4ull * ncd;
    if (ver == 1 && (ncd & 1)) q += 4;
    if (id != 1 && id != 2 && id != 3) fail("filter %d is not supported (deflate, shuffle, fletcher32 are)", id);
    ds.filters.push_back(id);
  }
}

// undo the pipeline (read order = reverse) on one chunk
std::vector<uint8_t> unfilter(const Dataset& ds, const uint8_t* src, uint64_t n, uint32_t mask,
                              uint64_t out_bytes) {
  std::vector<uint8_t> cur(src, src + n);
  for (int i = (int)ds.filters.size() - 1; i >= 0; --i) {
    if (mask & (1u << i)) continue;
    const int id = ds.filters[i];
    if (id == 1) {  // deflate
      std::vector<uint8_t> o(out_bytes);
      uLongf ol = (uLongf)out_bytes;
      const int rc = uncompress(o.data(), &ol, cur.data(), (uLong)cur.size());
      if (rc != Z_OK) fail("inflate failed (zlib %d)", rc);
      o.resize(ol);
      cur.swap(o);
    } else if (id == 2) {  // shuffle: byte planes -> elements
      const size_t es = (size_t)ds.esize, ne = cur.size() / es;
      std::vector<uint8_t> o(cur.size());
      for (size_t b = 0; b < es; ++b)
        for (size_t e = 0; e < ne; ++e) o[e * es + b] = cur[b * ne + e];
      std::memcpy(o.data() + ne * es, cur.data() + ne * es, cur.size() - ne * es);
      cur.swap(o);
    } else if (id == 3) {  // fletcher32: drop the trailing checksum
      if (cur.size() < 4) fail("fletcher32 chunk too short");
      cur.resize(cur.size() - 4);
    }
  }
  if (cur.size() < out_bytes) fail("chunk decodes to %zu bytes, %llu expected", cur.size(),
                                   (unsigned long long)out_bytes);
  return cur;
}

// copy a decoded chunk (chunk dims cd, at element offsets off) into ds.raw
void place_chunk(Dataset& ds, const std::vector<uint64_t>& cd, const std::vector<uint64_t>& off,
                 const uint8_t* data) {
  const int r = (int)ds.dims.size();
  const size_t es = ds.esize;
  std::vector<uint64_t> idx(r, 0);
  const uint64_t inner = cd[r - 1];
  while (true) {
    // one run along the last dimension
    bool inside = true;
    uint64_t dst = 0, srco = 0;
    for (int d = 0; d < r; ++d) {
      const uint64_t g = off[d] + idx[d];
      if (d < r - 1 && g >= ds.dims[d]) inside = false;
      dst = dst * ds.dims[d] + (d < r - 1 ? g : off[d]);
      srco = srco * cd[d] + (d < r - 1 ? idx[d] : 0);
    }
    if (inside && off[r - 1] < ds.dims[r - 1]) {
      const uint64_t nrun = std::min<uint64_t>(inner, ds.dims[r - 1] - off[r - 1]);
      std::memcpy(ds.raw.data() + dst * es, data + srco * es, nrun * es);
    }
    int d = r - 2;
    for (; d >= 0; --d) {
      if (++idx[d] < cd[d]) break;
      idx[d] = 0;
    }
    if (d < 0) break;
  }
}

void read_chunk(const File& f, Dataset& ds, const std::vector<uint64_t>& cd,
                const std::vector<uint64_t>& off, uint64_t a, uint64_t size, uint32_t mask) {
  if (a == UNDEF) return;  // never written: fill value (zero)
  const uint64_t cbytes = count(cd) * ds.esize;
  f.need(a, size);
  if (ds.filters.empty()) {
    if (size < cbytes) fail("short unfiltered chunk");
    place_chunk(ds, cd, off, f.p + a);
  } else {
    const std::vector<uint8_t> dec = unfilter(ds, f.p + a, size, mask, cbytes);
    place_chunk(ds, cd, off, dec.data());
  }
}

void read_btree_chunks(const File& f, Dataset& ds, uint64_t node, const std::vector<uint64_t>& cd) {
  const int r = (int)ds.dims.size();
  if (!f.sig(node, "TREE")) fail("bad chunk B-tree node");
  if (f.u(node + 4, 1) != 1) fail("chunk B-tree of type %d", (int)f.u(node + 4, 1));
  const int level = (int)f.u(node + 5, 1), used = (int)f.u(node + 6, 2);
  const uint64_t keysz = 8 + 8ull * (r + 1);
  uint64_t q = node + 8 + 2 * f.so;
  for (int i = 0; i < used; ++i) {
    const uint64_t size = f.u(q, 4);
    const uint32_t mask = (uint32_t)f.u(q + 4, 4);
    std::vector<uint64_t> off(r);
    for (int d = 0; d < r; ++d) off[d] = f.u(q + 8 + 8ull * d, 8);
    const uint64_t child = f.addr(q + keysz);
    if (level > 0) read_btree_chunks(f, ds, child, cd);
    else read_chunk(f, ds, cd, off, child, size, mask);
    q += keysz + f.so;
  }
}

// chunk offsets in row-major chunk order (implicit / fixed-array indexes)
std::vector<uint64_t> chunk_offset(const Dataset& ds, const std::vector<uint64_t>& cd, uint64_t k) {
  const int r = (int)ds.dims.size();
  std::vector<uint64_t> off(r);
  for (int d = r - 1; d >= 0; --d) {
    const uint64_t nc = (ds.dims[d] + cd[d] - 1) / cd[d];
    off[d] = (k % nc) * cd[d];
    k /= nc;
  }
  return off;
}

void read_layout(const File& f, const Msg& m, Dataset& ds) {
  const int ver = (int)f.u(m.off, 1);
  const uint64_t total = count(ds.dims) * ds.esize;
  ds.raw.assign(total, 0);
  const int r = (int)ds.dims.size();
  if (ver != 3 && ver != 4) fail("data layout message version %d", ver);
  const int klass = (int)f.u(m.off + 1, 1);
  if (klass == 0) {  // compact
    const uint64_t sz = f.u(m.off + 2, 2);
    f.need(m.off + 4, sz);
    std::memcpy(ds.raw.data(), f.p + m.off + 4, std::min(sz, total));
    return;
  }
  if (klass == 1) {  // contiguous
    const uint64_t a = f.addr(m.off + 2);
    if (a == UNDEF) return;
    f.need(a, total);
    std::memcpy(ds.raw.data(), f.p + a, total);
    return;
  }
  if (klass != 2) fail("layout class %d (virtual?) is not supported", klass);
  std::vector<uint64_t> cd(r);
  if (ver == 3) {
    const int nd = (int)f.u(m.off + 2, 1);  // rank + 1
    const uint64_t bt = f.addr(m.off + 3);
    for (int d = 0; d < r; ++d) cd[d] = f.u(m.off + 3 + f.so + 4ull * d, 4);
    (void)nd;
    if (bt != UNDEF) read_btree_chunks(f, ds, bt, cd);
    return;
  }
  // layout v4
  const int flags = (int)f.u(m.off + 2, 1), nd = (int)f.u(m.off + 3, 1), enc = (int)f.u(m.off + 4, 1);
  uint64_t q = m.off + 5;
  for (int d = 0; d < nd; ++d) {
    if (d < r) cd[d] = f.u(q, enc);
    q += enc;
  }
  const int itype = (int)f.u(q++, 1);
  const uint64_t cbytes = count(cd) * ds.esize;
  const uint64_t nchunks = [&] {
    uint64_t n = 1;
    for (int d = 0; d < r; ++d) n *= (ds.dims[d] + cd[d] - 1) / cd[d];
    return n;
  }();
  if (itype == 1) {  // single chunk
    uint64_t size = cbytes;
    uint32_t mask = 0;
    if (flags & 2) {
      size = f.len(q);
      mask = (uint32_t)f.u(q + f.sl, 4);
      q += f.sl + 4;
    }
    read_chunk(f, ds, cd, std::vector<uint64_t>(r, 0), f.addr(q), size, mask);
  } else if (itype == 2) {  // implicit: chunks stored in order, unfiltered
    const uint64_t a = f.addr(q);
    for (uint64_t k = 0; k < nchunks && a != UNDEF; ++k)
      read_chunk(f, ds, cd, chunk_offset(ds, cd, k), a + k * cbytes, cbytes, 0);
  } else if (itype == 3) {  // fixed array
    q += 1;                 // page bits
    const uint64_t hdr = f.addr(q);
    if (hdr == UNDEF) return;
    if (!f.sig(hdr, "FAHD")) fail("bad fixed-array header");
    const int client = (int)f.u(hdr + 5, 1), elsz = (int)f.u(hdr + 6, 1), pbits = (int)f.u(hdr + 7, 1);
    const uint64_t nel = f.len(hdr + 8);
    if (nel > (1ull << pbits)) fail("paged fixed-array chunk index is not supported");
    const uint64_t db = f.addr(hdr + 8 + f.sl);
    if (!f.sig(db, "FADB")) fail("bad fixed-array data block");
    uint64_t e = db + 6 + f.so;
    for (uint64_t k = 0; k < nel && k < nchunks; ++k) {
      const uint64_t a = f.addr(e);
      uint64_t size = cbytes;
      uint32_t mask = 0;
      if (client == 1) {
        const int szlen = elsz - f.so - 4;
        size = f.u(e + f.so, szlen);
        mask = (uint32_t)f.u(e + f.so + szlen, 4);
      }
      read_chunk(f, ds, cd, chunk_offset(ds, cd, k), a, size, mask);
      e += elsz;
    }
  } else {
    fail("chunk index type %d (extensible array / v2 B-tree) is not supported", itype);
  }
}

void open_file(File& f, const char* path) {
  f.fd = open(path, O_RDONLY);
  if (f.fd < 0) fail("cannot open %s", path);
  struct stat st;
  if (fstat(f.fd, &st) != 0) fail("cannot stat %s", path);
  f.n = (size_t)st.st_size;
  void* m = mmap(nullptr, f.n, PROT_READ, MAP_PRIVATE, f.fd, 0);
  if (m == MAP_FAILED) fail("cannot map %s", path);
  f.p = static_cast<const uint8_t*>(m);
  static const uint8_t magic[8] = {0x89, 'H', 'D', 'F', '\r', '\n', 0x1a, '\n'};
  if (f.n < 64 || std::memcmp(f.p, magic, 8) != 0) fail("%s: not an HDF5 file (no signature at 0)", path);
}

uint64_t root_group(File& f) {
  const int ver = (int)f.u(8, 1);
  if (ver == 0 || ver == 1) {
    f.so = (int)f.u(13, 1);
    f.sl = (int)f.u(14, 1);
    const uint64_t q = ver == 0 ? 24 : 28;
    f.base = f.u(q, f.so);
    const uint64_t entry = q + 4ull * f.so;  // root group symbol table entry
    return f.addr(entry + f.so);
  }
  if (ver == 2 || ver == 3) {
    f.so = (int)f.u(9, 1);
    f.sl = (int)f.u(10, 1);
    f.base = f.u(12, f.so);
    return f.addr(12 + 3ull * f.so);
  }
  fail("superblock version %d", ver);
}

Dataset load(const char* path, const char* name, bool with_data) {
  File f;
  open_file(f, path);
  uint64_t oh = root_group(f);
  std::string rest(name);
  while (!rest.empty() && rest[0] == '/') rest.erase(0, 1);
  while (!rest.empty()) {
    const size_t s = rest.find('/');
    const std::string part = rest.substr(0, s);
    oh = lookup(f, oh, part);
    if (oh == UNDEF) fail("%s: no object '%s'", path, name);
    rest = s == std::string::npos ? "" : rest.substr(s + 1);
  }
  const std::vector<Msg> ms = object_messages(f, oh);
  const Msg* sp = find(ms, 0x01);
  const Msg* ty = find(ms, 0x03);
  const Msg* lay = find(ms, 0x08);
  if (!sp || !ty || !lay) fail("%s: '%s' is not a dataset", path, name);
  Dataset ds;
  parse_dataspace(f, *sp, ds);
  parse_datatype(f, *ty, ds);
  if (const Msg* fl = find(ms, 0x0B)) parse_filters(f, *fl, ds);
  if (find(ms, 0x07)) fail("external storage is not supported");
  if (with_data) read_layout(f, *lay, ds);
  return ds;
}

template <typename T>
T element(const Dataset& ds, uint64_t i) {
  uint8_t b[8];
  std::memcpy(b, ds.raw.data() + i * ds.esize, ds.esize);
  if (ds.big_endian)
    for (int k = 0; k < ds.esize / 2; ++k) std::swap(b[k], b[ds.esize - 1 - k]);
  if (ds.klass == 1) {
    if (ds.esize == 4) {
      float v;
      std::memcpy(&v, b, 4);
      return (T)v;
    }
    double v;
    std::memcpy(&v, b, 8);
    return (T)v;
  }
  uint64_t u = 0;
  for (int k = ds.esize - 1; k >= 0; --k) u = (u << 8) | b[k];
  if (ds.is_signed && ds.esize < 8 && (u >> (8 * ds.esize - 1)) & 1) u |= ~0ull << (8 * ds.esize);
  return ds.is_signed ? (T)(int64_t)u : (T)u;
}

}  // namespace

extern "C" {

int pcadv_h5_info(const char* path, const char* name, int* rank, int64_t* dims, int* dtype) {
  try {
    if (!path || !name || !rank || !dims || !dtype) fail("h5_info: null argument");
    const Dataset ds = load(path, name, false);
    if (ds.dims.size() > 8) fail("rank %zu > 8", ds.dims.size());
    *rank = (int)ds.dims.size();
    for (size_t i = 0; i < ds.dims.size(); ++i) dims[i] = (int64_t)ds.dims[i];
    *dtype = ds.klass == 1 ? (ds.esize == 4 ? PCADV_H5_F32 : PCADV_H5_F64)
                           : (ds.is_signed ? PCADV_H5_INT : PCADV_H5_UINT) | (ds.esize << 4);
    return PCADV_OK;
  } catch (const H5Error& e) {
    pcadv::set_error("%s", e.msg.c_str());
    return PCADV_EINVAL;
  } catch (const std::bad_alloc&) {
    pcadv::set_error("h5: out of host memory");
    return PCADV_EINVAL;
  }
}

int pcadv_h5_read(const char* path, const char* name, int out_type, int64_t keep1, void* out,
                  size_t out_bytes) {
  try {
    if (!path || !name || !out) fail("h5_read: null argument");
    if (out_type != PCADV_H5_OUT_F32 && out_type != PCADV_H5_OUT_I64) fail("h5_read: out_type %d", out_type);
    const Dataset ds = load(path, name, true);
    const int r = (int)ds.dims.size();
    std::vector<uint64_t> od = ds.dims;
    if (r >= 2 && keep1 > 0 && (uint64_t)keep1 < od[1]) od[1] = (uint64_t)keep1;
    const uint64_t n = count(od);
    const size_t es = out_type == PCADV_H5_OUT_F32 ? 4 : 8;
    if (out_bytes < n * es) fail("h5_read: output holds %zu bytes, %llu needed", out_bytes,
                                 (unsigned long long)(n * es));
    // rows of the leading dimension; dim 1 cut to od[1] (data[:, 0:npts, ...])
    const uint64_t inner = r >= 3 ? count(std::vector<uint64_t>(ds.dims.begin() + 2, ds.dims.end())) : 1;
    const uint64_t rows = r >= 1 ? ds.dims[0] : 1;
    const uint64_t d1 = r >= 2 ? ds.dims[1] : 1, k1 = r >= 2 ? od[1] : 1;
    uint64_t o = 0;
    for (uint64_t a = 0; a < rows; ++a)
      for (uint64_t b = 0; b < k1; ++b)
        for (uint64_t c = 0; c < inner; ++c, ++o) {
          const uint64_t i = (a * d1 + b) * inner + c;
          if (out_type == PCADV_H5_OUT_F32) static_cast<float*>(out)[o] = element<float>(ds, i);
          else static_cast<int64_t*>(out)[o] = element<int64_t>(ds, i);
        }
    return PCADV_OK;
  } catch (const H5Error& e) {
    pcadv::set_error("%s", e.msg.c_str());
    return PCADV_EINVAL;
  } catch (const std::bad_alloc&) {
    pcadv::set_error("h5: out of host memory");
    return PCADV_EINVAL;
  }
}

}  // extern "C"
