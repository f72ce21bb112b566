// CPU harness for the device physics (TEST ONLY).  Compiles the product source
// (csrc/fw_kernels.hip) and runs its __host__ __device__ per-aircraft functions
// on the host, so tests can compare the exact kernel code paths with the
// independent oracle without a GPU.  Never loaded by the product.
#include "../../tum_adlr_deep_reinforcement_learning_amd/csrc/fw_kernels.hip"

template <typename T>
static void run_sim(const fw_sim_config* sc, int64_t n, const double* y_in, const double* der_in, const double* wind,
                    const double* turb, const double* cmd_in, double* y_out, double* der_out, double* cmd_out,
                    int32_t* term, int32_t* nfev, int32_t* nacc) {
  fw_handle h;
  h.sim = *sc;
  h.has_env = false;
  DevCfg<T> d;
  fill_devcfg(&h, d);
  for (int64_t i = 0; i < n; i++) {
    T y[FW_NY], der[8], cmd[3], w[3], tl[3], ta[3];
    for (int k = 0; k < FW_NY; k++) y[k] = (T)y_in[i * FW_NY + k];
    for (int k = 0; k < 8; k++) der[k] = (T)der_in[i * 8 + k];
    for (int k = 0; k < 3; k++) {
      cmd[k] = (T)cmd_in[i * 3 + k];
      w[k] = (T)wind[i * 3 + k];
      tl[k] = (T)turb[i * 6 + k];
      ta[k] = (T)turb[i * 6 + 3 + k];
    }
    int nf = 0, na = 0;
    uint32_t dm = 0;
    fw::V2<T> sy[fw::NP], sf[2 * fw::NP];  // sf + NP: error-sum slots when FW_ER_LDS
    term[i] = sim_step_masked<1, false, T>(d, d, y, der, cmd, w, tl, ta, nf, na, dm, sy, sf, 1);
    nfev[i] = nf;
    nacc[i] = na;
    for (int k = 0; k < FW_NY; k++) y_out[i * FW_NY + k] = (double)y[k];
    for (int k = 0; k < 8; k++) der_out[i * 8 + k] = (dm >> k) & 1 ? (double)der[k] : der_in[i * 8 + k];
    for (int k = 0; k < 3; k++) cmd_out[i * 3 + k] = (double)cmd[k];
  }
}

extern "C" void fwt_sim_step(int32_t precision, const fw_sim_config* sc, int64_t n, const double* y_in,
                             const double* der_in, const double* wind, const double* turb, const double* cmd_in,
                             double* y_out, double* der_out, double* cmd_out, int32_t* term, int32_t* nfev,
                             int32_t* nacc) {
  if (precision == FW_F64)
    run_sim<double>(sc, n, y_in, der_in, wind, turb, cmd_in, y_out, der_out, cmd_out, term, nfev, nacc);
  else
    run_sim<float>(sc, n, y_in, der_in, wind, turb, cmd_in, y_out, der_out, cmd_out, term, nfev, nacc);
}

extern "C" void fwt_reset_derived(const fw_sim_config* sc, const double* y, const double* euler, const double* wind,
                                  double* der) {
  fw_handle h;
  h.sim = *sc;
  DevCfg<double> d;
  fill_devcfg(&h, d);
  double dd[8] = {euler[0], euler[1], euler[2], 0, 0, 0, 0, 0};
  reset_derived<double>(d, y, wind, dd);
  for (int k = 0; k < 8; k++) der[k] = dd[k];
}

extern "C" void fwt_philox(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                           uint32_t* out) {
  philox(k0, k1, c0, c1, c2, c3, out);
}
