// The xGMI link-check verdict of `gpu-burnin --p2p` (the SSH / Terraform path), in one
// place: the same rules as node/labels.py:link_labels (the node agent's path), which
// tests/test_link_verdict.py holds it to over generated matrices.  Host code only.
//
// mat[i*n+j]: GB/s of the transfer i -> j (< 0: it failed); acc[i*n+j]: j could map i's
// memory; derr[i*n+j]: mismatching words of what arrived (> 0: the link corrupted data).
// A pair is degraded below min_frac of the node's median, below the absolute floor
// min_gbps (a uniformly slow fabric has a healthy-looking median), or when its data was
// wrong.  A pair that failed, or that was measured without peer access, makes the node's
// status "error".
#pragma once

#include <algorithm>
#include <vector>

struct TkLinkVerdict {
  int measured = 0, degraded = 0, below_floor = 0, corrupt = 0, errors = 0, no_peer = 0;
  double min_gbps = 0.0, median_gbps = 0.0;
  const char* status = "error";
};

inline double tk_median(std::vector<double> v) {
  if (v.empty()) return 0.0;
  std::sort(v.begin(), v.end());
  const size_t m = v.size();
  return m % 2 ? v[m / 2] : 0.5 * (v[m / 2 - 1] + v[m / 2]);
}

inline TkLinkVerdict tk_link_verdict(int n, const double* mat, const int* acc, const double* derr, double min_frac,
                                     double min_gbps) {
  TkLinkVerdict v;
  std::vector<double> vals;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      if (i == j) continue;
      if (mat[i * n + j] < 0.0) {
        ++v.errors;
        continue;
      }
      if (!acc[i * n + j]) ++v.no_peer;
      vals.push_back(mat[i * n + j]);
    }
  v.measured = (int)vals.size();
  v.median_gbps = tk_median(vals);
  v.min_gbps = vals.empty() ? 0.0 : *std::min_element(vals.begin(), vals.end());
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      if (i == j || mat[i * n + j] < 0.0) continue;
      const double g = mat[i * n + j];
      const bool bad_data = derr[i * n + j] > 0.0;
      v.degraded += g < min_frac * v.median_gbps || g < min_gbps || bad_data;
      v.below_floor += g < min_gbps;
      v.corrupt += bad_data;
    }
  v.status = (v.errors || v.no_peer || v.measured == 0) ? "error" : (v.degraded ? "degraded" : "passed");
  return v;
}

// The matrix's only fault is speed: it is worth measuring again (best of up to 3 per pair,
// node/labels.py:best_link_verdict).  A pair that failed, lacked peer access or delivered
// wrong data is never retried away.
inline bool tk_link_slow_only(int n, const double* mat, const int* acc, const double* derr, double min_frac,
                              double min_gbps) {
  const TkLinkVerdict v = tk_link_verdict(n, mat, acc, derr, min_frac, min_gbps);
  return v.errors == 0 && v.no_peer == 0 && v.corrupt == 0 && v.measured > 0 && v.degraded > 0;
}
