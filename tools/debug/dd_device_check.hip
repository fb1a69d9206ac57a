// Debug harness (not part of libsid): double-double log and the -m local fast
// path evaluated on the device vs the host, for near-tie profiles.
#include "../../sid_amd/csrc/local.hip"
#include <cstdio>
#include <vector>
#include <cmath>

__global__ void k_dd(const double* xs, int n, double* out) {
  int i = threadIdx.x; if (i >= n) return;
  sid_dd r = dd_log(xs[i]); out[2*i] = r.hi; out[2*i+1] = r.lo;
}
__global__ void k_fast(sid_local_k K, const double* lnt, const unsigned* c, int n, double* out) {
  int i = threadIdx.x; if (i >= n) return;
  double p1, p2; bool gt;
  bool ok = local_fast_p(c[3*i], c[3*i+1], c[3*i+2], K, lnt, p1, p2, gt);
  out[4*i] = ok; out[4*i+1] = p1; out[4*i+2] = p2;
  out[4*i+3] = sid_local_refine_d(c[3*i], c[3*i+1], c[3*i+2], K.E, 0, 0);
}
int main() {
  std::vector<double> xs = {0.25, 0.1, 1.0/3.0, 0.9, 1e-300, 0.5833333333333334};
  double *dx, *dout; hipMalloc(&dx, 64*8); hipMalloc(&dout, 256*8);
  hipMemcpy(dx, xs.data(), xs.size()*8, hipMemcpyHostToDevice);
  k_dd<<<1,64>>>(dx, xs.size(), dout);
  std::vector<double> o(256); hipMemcpy(o.data(), dout, 256*8, hipMemcpyDeviceToHost);
  for (size_t i = 0; i < xs.size(); ++i) { sid_dd h = dd_log(xs[i]);
    printf("dd_log %.17g dev %.17g %.17g host %.17g %.17g\n", xs[i], o[2*i], o[2*i+1], h.hi, h.lo); }
  sid_local_k K{}; K.E = 2.0; K.sig = 0.05; K.cA1 = std::log(1-2.0); K.cB1 = std::log(2.0/3.);
  K.cA2 = std::log((1-2./3.*2.0)/2.); K.cB2 = K.cB1; K.prior = -1; K.lg15 = -0.12078223763524432;
  std::vector<double> lnt(SID_LUTN); lnt[0] = -INFINITY; for (int k = 1; k < SID_LUTN; ++k) lnt[k] = std::log((double)k);
  double* dl; hipMalloc(&dl, SID_LUTN*8); hipMemcpy(dl, lnt.data(), SID_LUTN*8, hipMemcpyHostToDevice);
  unsigned cs[] = {1,1,2, 3,3,6, 2,2,4, 20,5,3};
  unsigned* dc; hipMalloc(&dc, sizeof cs); hipMemcpy(dc, cs, sizeof cs, hipMemcpyHostToDevice);
  k_fast<<<1,64>>>(K, dl, dc, 4, dout); hipMemcpy(o.data(), dout, 256*8, hipMemcpyDeviceToHost);
  for (int i = 0; i < 4; ++i) { double p1, p2; bool gt; bool ok = local_fast_p(cs[3*i], cs[3*i+1], cs[3*i+2], K, lnt.data(), p1, p2, gt);
    printf("fast %u %u %u dev ok=%g p1=%.17g p2=%.17g refine=%.17g | host ok=%d p1=%.17g p2=%.17g refine=%.17g\n",
      cs[3*i], cs[3*i+1], cs[3*i+2], o[4*i], o[4*i+1], o[4*i+2], o[4*i+3], ok, p1, p2, sid_local_refine_d(cs[3*i], cs[3*i+1], cs[3*i+2], 2.0, 0, 0)); }
  return 0;
}
