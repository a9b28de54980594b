// buckets.cpp — see buckets.h.
#include "buckets.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <map>

namespace dg {

std::string aspect_ratio_to_str(uint32_t w, uint32_t h) {
  // Rust "{:.3}" prints the correctly rounded decimal of the exact binary
  // value; glibc printf does the same.
  char buf[64];
  snprintf(buf, sizeof(buf), "%.3f", (double)w / (double)h);
  return std::string(buf);
}

std::vector<std::pair<uint32_t, uint32_t>> build_image_size_list(uint32_t default_image_size,
                                                                 uint32_t downsampling_ratio,
                                                                 double min_ar, double max_ar) {
  std::vector<std::pair<uint32_t, uint32_t>> out;
  uint32_t patch = default_image_size / downsampling_ratio;
  double patch_sq = (double)(uint32_t)(patch * patch);
  uint32_t min_pw = (uint32_t)ceil(sqrt(patch_sq * min_ar));
  uint32_t max_pw = (uint32_t)floor(sqrt(patch_sq * max_ar));
  for (uint32_t pw = min_pw; pw <= max_pw && pw != 0; pw++) {
    uint32_t ph = (uint32_t)floor(patch_sq / (double)pw);
    out.emplace_back(pw * downsampling_ratio, ph * downsampling_ratio);
  }
  uint32_t min_ph = (uint32_t)ceil(sqrt(patch_sq / max_ar));
  uint32_t max_ph = (uint32_t)floor(sqrt(patch_sq / min_ar));
  for (uint32_t ph = min_ph; ph <= max_ph && ph != 0; ph++) {
    uint32_t pw = (uint32_t)floor(patch_sq / (double)ph);
    out.emplace_back(pw * downsampling_ratio, ph * downsampling_ratio);
  }
  return out;
}

BucketTable::BucketTable(uint32_t default_image_size, uint32_t downsampling_ratio, double min_ar,
                         double max_ar) {
  sizes_ = build_image_size_list(default_image_size, downsampling_ratio, min_ar, max_ar);
  // HashMap insert: last insert wins per key (image_processing.rs:104-108)
  std::map<std::string, std::pair<uint32_t, uint32_t>> m;
  for (auto &s : sizes_) m[aspect_ratio_to_str(s.first, s.second)] = s;
  for (auto &kv : m) sorted_.push_back(Bucket{strtod(kv.first.c_str(), nullptr), kv.first, kv.second.first, kv.second.second});
  std::stable_sort(sorted_.begin(), sorted_.end(), [](const Bucket &a, const Bucket &b) { return a.ar < b.ar; });
}

int BucketTable::closest(int32_t w, int32_t h) const {
  if (sorted_.empty()) return -1;
  double t = (double)w / (double)h;
  // binary_search_by(partial_cmp): Ok(idx) on exact match, Err(insertion point)
  size_t lo = 0, hi = sorted_.size();
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    if (sorted_[mid].ar < t) lo = mid + 1;
    else hi = mid;
  }
  size_t idx = lo;
  if (idx < sorted_.size() && sorted_[idx].ar == t) return (int)idx;
  if (idx == 0) return 0;
  if (idx == sorted_.size()) return (int)sorted_.size() - 1;
  double left = fabs(t - sorted_[idx - 1].ar);
  double right = fabs(sorted_[idx].ar - t);
  return left < right ? (int)idx - 1 : (int)idx;  // ties go right
}

int BucketTable::find_key(const std::string &key) const {
  for (size_t i = 0; i < sorted_.size(); i++)
    if (sorted_[i].key == key) return (int)i;
  return -1;
}

double rust_round(double x) { return x >= 0 ? floor(x + 0.5) : -floor(-x + 0.5); }

void scaled_size(uint32_t w, uint32_t h, uint32_t tw, uint32_t th, uint32_t &nw, uint32_t &nh) {
  double sx = (double)tw / (double)w, sy = (double)th / (double)h;
  double s = sx > sy ? sx : sy;  // f64::max
  nw = (uint32_t)rust_round((double)w * s);
  nh = (uint32_t)rust_round((double)h * s);
}

void fit_crop_box(uint32_t sw, uint32_t sh, uint32_t dw, uint32_t dh, double &l, double &t, double &cw,
                  double &ch) {
  if (!sw || !sh || !dw || !dh) {
    l = t = 0;
    cw = sw;
    ch = sh;
    return;
  }
  double width = sw, height = sh;
  double ir = width / height, rr = (double)dw / (double)dh;
  if (fabs(ir - rr) < 2.220446049250313e-16) {
    cw = width;
    ch = height;
  } else if (ir >= rr) {
    cw = rr * height;
    ch = height;
  } else {
    cw = width;
    ch = width / rr;
  }
  l = (width - cw) * 0.5;
  t = (height - ch) * 0.5;
}

}  // namespace dg
