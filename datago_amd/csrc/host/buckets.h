// buckets.h — aspect-ratio bucket table (product C++).
// Reference: /root/reference/src/image_processing.rs
//   get_ar_aware_transform :77-121, aspect_ratio_to_str :130-133,
//   build_image_size_list :188-219, get_closest_aspect_ratio :222-252,
//   scale/round :278-286, and fast_image_resize CropBox::fit_src_into_dst_size
//   (called at :304-310).
#pragma once
#include <stdint.h>

#include <string>
#include <utility>
#include <vector>

namespace dg {

struct Bucket {
  double ar;         // parsed key
  std::string key;   // "%.3f"
  uint32_t w, h;
};

class BucketTable {
 public:
  BucketTable(uint32_t default_image_size, uint32_t downsampling_ratio, double min_ar, double max_ar);
  int closest(int32_t w, int32_t h) const;        // index into sorted buckets
  int find_key(const std::string &key) const;     // -1 if absent
  const std::vector<Bucket> &buckets() const { return sorted_; }
  const std::vector<std::pair<uint32_t, uint32_t>> &size_list() const { return sizes_; }

 private:
  std::vector<std::pair<uint32_t, uint32_t>> sizes_;
  std::vector<Bucket> sorted_;
};

std::string aspect_ratio_to_str(uint32_t w, uint32_t h);
std::vector<std::pair<uint32_t, uint32_t>> build_image_size_list(uint32_t default_image_size,
                                                                 uint32_t downsampling_ratio,
                                                                 double min_ar, double max_ar);
double rust_round(double x);
void scaled_size(uint32_t w, uint32_t h, uint32_t tw, uint32_t th, uint32_t &nw, uint32_t &nh);
void fit_crop_box(uint32_t sw, uint32_t sh, uint32_t dw, uint32_t dh, double &l, double &t, double &cw,
                  double &ch);

}  // namespace dg
