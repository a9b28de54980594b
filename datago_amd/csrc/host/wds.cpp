// wds.cpp — WebDataset shard indexing on the host.
//
// Replaces the tar walk of pull_tarballs (reference generator_wds.rs:56-204,
// async-tar 0.5 / tar 0.4): every regular-file entry of the shard, its
// sample key = Path::file_stem of the entry path (the basename without its
// last extension), rank filtering by DefaultHasher (SipHash-1-3, keys 0/0)
// of the key % world_size (:50-54, :133-148), consecutive entries of equal
// key grouped into one sample, reference extension first (stable, :154-166).
// Zero-copy: members are (offset, length) pairs into the caller's shard
// buffer, so their bytes go straight to dg_submit (or, with the shard
// uploaded to HBM once, to dg_submit_device).
#include <string.h>

#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/datago_hip.h"

namespace dg {
void set_error(const std::string &s);

static inline uint64_t rotl(uint64_t x, int b) { return (x << b) | (x >> (64 - b)); }

// SipHash-1-3 with k0 = k1 = 0 of (bytes, 0xFF): Rust's DefaultHasher over a &str.
uint64_t siphash13_str(const uint8_t *p, size_t n) {
  uint64_t v0 = 0x736F6D6570736575ull, v1 = 0x646F72616E646F6Dull, v2 = 0x6C7967656E657261ull,
           v3 = 0x7465646279746573ull;
  auto round = [&]() {
    v0 += v1; v1 = rotl(v1, 13); v1 ^= v0; v0 = rotl(v0, 32);
    v2 += v3; v3 = rotl(v3, 16); v3 ^= v2;
    v0 += v3; v3 = rotl(v3, 21); v3 ^= v0;
    v2 += v1; v1 = rotl(v1, 17); v1 ^= v2; v2 = rotl(v2, 32);
  };
  const size_t total = n + 1;  // the 0xFF terminator of str::hash
  auto byte = [&](size_t i) -> uint64_t { return i < n ? p[i] : 0xFFu; };
  size_t i = 0;
  for (; i + 8 <= total; i += 8) {
    uint64_t m = 0;
    for (int k = 0; k < 8; k++) m |= byte(i + k) << (8 * k);
    v3 ^= m;
    round();
    v0 ^= m;
  }
  uint64_t b = (uint64_t)(total & 0xFF) << 56;
  for (size_t k = 0; i + k < total; k++) b |= byte(i + k) << (8 * k);
  v3 ^= b;
  round();
  v0 ^= b;
  v2 ^= 0xFF;
  round();
  round();
  round();
  return v0 ^ v1 ^ v2 ^ v3;
}

namespace {
uint64_t octal(const uint8_t *f, size_t n, bool &ok) {
  if (f[0] & 0x80) {  // GNU base-256 (two's complement, big-endian; tar 0.4 rejects what does not fit u64)
    if (f[0] & 0x40) {  // negative
      ok = false;
      return 0;
    }
    uint64_t v = f[0] & 0x3F;
    for (size_t i = 1; i < n; i++) {
      if (v >> 56) {  // would overflow 64 bits
        ok = false;
        return 0;
      }
      v = (v << 8) | f[i];
    }
    return v;
  }
  uint64_t v = 0;
  size_t i = 0;
  while (i < n && (f[i] == ' ' || f[i] == 0)) i++;
  for (; i < n && f[i] >= '0' && f[i] <= '7'; i++) v = v * 8 + (uint64_t)(f[i] - '0');
  for (; i < n; i++)
    if (f[i] != ' ' && f[i] != 0) ok = false;
  return v;
}

std::string cstr(const uint8_t *f, size_t n) {
  size_t k = 0;
  while (k < n && f[k]) k++;
  return std::string((const char *)f, k);
}

// pax records "len key=value\n"
bool pax_path(const uint8_t *d, size_t n, std::string &path) {
  size_t i = 0;
  bool found = false;
  while (i < n) {
    size_t j = i, len = 0;
    while (j < n && d[j] >= '0' && d[j] <= '9' && len <= n) len = len * 10 + (d[j++] - '0');
    // a record holds at least its length digits, the space and the trailing newline
    if (j >= n || d[j] != ' ' || len < (j + 1 - i) + 1 || len > n - i) break;
    const std::string rec((const char *)d + j + 1, len - (j + 1 - i) - 1);
    const size_t eq = rec.find('=');
    if (eq != std::string::npos && rec.compare(0, eq, "path") == 0) {
      path = rec.substr(eq + 1);
      found = true;
    }
    i += len;
  }
  return found;
}

// Path::file_stem: the last component without its last extension ("a.b.jpg" -> "a.b",
// ".hidden" -> ".hidden", "x." -> "x")
std::string file_stem(const std::string &p) {
  size_t e = p.size();
  while (e > 0 && p[e - 1] == '/') e--;
  const std::string t = p.substr(0, e);
  const size_t sl = t.rfind('/');
  const std::string base = sl == std::string::npos ? t : t.substr(sl + 1);
  if (base == "..") return base;
  const size_t dot = base.rfind('.');
  if (dot == std::string::npos || dot == 0) return base;
  return base.substr(0, dot);
}

}  // namespace

}  // namespace dg

extern "C" {

uint64_t dg_wds_key_hash(const char *key, size_t len) { return dg::siphash13_str((const uint8_t *)key, len); }

static dg_status wds_index_impl(const uint8_t *tar, size_t len, int32_t rank, int32_t world_size,
                                const char *reference_ext, dg_wds_member *members, int64_t mcap, int64_t *nmembers,
                                char *names, size_t ncap, size_t *nnames, dg_wds_sample *samples, int64_t scap,
                                int64_t *nsamples) {
  if (!tar || !nmembers || !nsamples || !nnames || world_size < 0 || (world_size > 1 && (rank < 0 || rank >= world_size)))
    return DG_ERR_INVALID;
  struct M {
    std::string name, key;
    uint64_t off, n;
  };
  std::vector<M> all;
  size_t pos = 0;
  std::string longname;
  bool have_long = false;
  while (pos + 512 <= len) {
    const uint8_t *h = tar + pos;
    bool zero = true;
    for (int i = 0; i < 512 && zero; i++) zero = h[i] == 0;
    if (zero) break;  // end of archive
    bool ok = true;
    const uint64_t size = dg::octal(h + 124, 12, ok);
    uint64_t chk = 0, want = dg::octal(h + 148, 8, ok);
    for (int i = 0; i < 512; i++) chk += (i >= 148 && i < 156) ? ' ' : h[i];
    if (!ok || chk != want) {
      dg::set_error("wds: bad tar header checksum");
      return DG_ERR_CORRUPT;
    }
    const uint64_t data = pos + 512;
    if (size > len - data) {  // data <= len here; never form data + size (it can wrap)
      dg::set_error("wds: truncated tar entry");
      return DG_ERR_CORRUPT;
    }
    const uint8_t type = h[156];
    if (type == 'L') {  // GNU long name: the next entry's path
      longname = dg::cstr(tar + data, (size_t)size);
      have_long = true;
    } else if (type == 'x') {  // pax extended header
      std::string p;
      if (dg::pax_path(tar + data, (size_t)size, p)) {
        longname = p;
        have_long = true;
      }
    } else if (type == 'g') {
      // global pax header: no per-entry path
    } else {
      std::string name;
      if (have_long) {
        name = longname;
      } else {
        name = dg::cstr(h, 100);
        const bool ustar = memcmp(h + 257, "ustar", 5) == 0;
        const std::string prefix = ustar ? dg::cstr(h + 345, 155) : std::string();
        if (!prefix.empty()) name = prefix + "/" + name;
      }
      have_long = false;
      if (type == '0' || type == 0 || type == '7') {
        const std::string key = dg::file_stem(name);
        if (world_size <= 1 || dg::siphash13_str((const uint8_t *)key.data(), key.size()) % (uint64_t)world_size ==
                                   (uint64_t)rank)
          all.push_back({name, key, data, size});
      }
    }
    pos = data + (size + 511) / 512 * 512;
  }
  // group consecutive equal keys; the reference extension first (stable)
  const std::string ref = reference_ext ? reference_ext : "";
  std::vector<size_t> order;
  std::vector<dg_wds_sample> groups;
  for (size_t i = 0; i < all.size();) {
    size_t j = i;
    while (j < all.size() && all[j].key == all[i].key) j++;
    const uint32_t first = (uint32_t)order.size();
    for (size_t k = i; k < j; k++)
      if (!ref.empty() && all[k].name.size() >= ref.size() &&
          all[k].name.compare(all[k].name.size() - ref.size(), ref.size(), ref) == 0)
        order.push_back(k);
    for (size_t k = i; k < j; k++)
      if (ref.empty() || !(all[k].name.size() >= ref.size() &&
                           all[k].name.compare(all[k].name.size() - ref.size(), ref.size(), ref) == 0))
        order.push_back(k);
    groups.push_back({first, (uint32_t)(j - i)});
    i = j;
  }
  size_t nb = 0;
  for (size_t k : order) nb += all[k].name.size() + 1;
  *nmembers = (int64_t)order.size();
  *nsamples = (int64_t)groups.size();
  *nnames = nb;
  if (!members || !samples || !names || (int64_t)order.size() > mcap || (int64_t)groups.size() > scap || nb > ncap) {
    dg::set_error("wds: output arrays too small (sizes reported)");
    return DG_ERR_SMALL_BUFFER;
  }
  size_t no = 0;
  for (size_t m = 0; m < order.size(); m++) {
    const M &e = all[order[m]];
    members[m].data_off = e.off;
    members[m].data_len = e.n;
    members[m].name_off = no;
    members[m].name_len = (uint32_t)e.name.size();
    members[m].pad = 0;
    memcpy(names + no, e.name.c_str(), e.name.size() + 1);
    no += e.name.size() + 1;
  }
  memcpy(samples, groups.data(), groups.size() * sizeof(dg_wds_sample));
  return DG_OK;
}

// No C++ exception may cross the C ABI (the Rust caller would abort): a
// malformed shard that trips one (e.g. an allocation for a hostile length)
// reports DG_ERR_CORRUPT like any other bad header.
dg_status dg_wds_index(const uint8_t *tar, size_t len, int32_t rank, int32_t world_size, const char *reference_ext,
                       dg_wds_member *members, int64_t mcap, int64_t *nmembers, char *names, size_t ncap,
                       size_t *nnames, dg_wds_sample *samples, int64_t scap, int64_t *nsamples) {
  try {
    return wds_index_impl(tar, len, rank, world_size, reference_ext, members, mcap, nmembers, names, ncap, nnames,
                          samples, scap, nsamples);
  } catch (const std::bad_alloc &) {
    dg::set_error("wds: out of host memory");
    return DG_ERR_OOM;
  } catch (const std::exception &e) {
    dg::set_error(std::string("wds: malformed shard (") + e.what() + ")");
    return DG_ERR_CORRUPT;
  }
}

}  // extern "C"
