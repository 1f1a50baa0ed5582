// Which hipBLASLt epilogues have solutions on this GPU for the GPT-2 345M MLP shapes?
// Heuristic queries only (no GEMM is run). Build + run on the GPU box:
//   hipcc -O2 scripts/probe_blaslt_epilogue.cpp -lhipblaslt -o /tmp/probe && /tmp/probe
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdio>

struct Epi {
  const char* name;
  hipblasLtEpilogue_t e;
  bool aux, bias;
};

int main() {
  hipblasLtHandle_t h;
  if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) {
    printf("hipblasLtCreate failed\n");
    return 1;
  }
  const Epi eps[] = {
      {"DEFAULT", HIPBLASLT_EPILOGUE_DEFAULT, false, false},
      {"BIAS", HIPBLASLT_EPILOGUE_BIAS, false, true},
      {"GELU", HIPBLASLT_EPILOGUE_GELU, false, false},
      {"GELU_BIAS", HIPBLASLT_EPILOGUE_GELU_BIAS, false, true},
      {"GELU_AUX", HIPBLASLT_EPILOGUE_GELU_AUX, true, false},
      {"GELU_AUX_BIAS", HIPBLASLT_EPILOGUE_GELU_AUX_BIAS, true, true},
      {"DGELU", HIPBLASLT_EPILOGUE_DGELU, true, false},
      {"DGELU_BGRAD", HIPBLASLT_EPILOGUE_DGELU_BGRAD, true, true},
      {"BGRADA", HIPBLASLT_EPILOGUE_BGRADA, false, true},
      {"BGRADB", HIPBLASLT_EPILOGUE_BGRADB, false, true},
  };
  const hipblasOperation_t ops[2] = {HIPBLAS_OP_N, HIPBLAS_OP_T};
  const char* opn[2] = {"N", "T"};
  const int aux_types[3] = {-1, (int)HIP_R_16BF, (int)HIP_R_32F};  // -1: attribute not set
  const hipDataType bias_types[2] = {HIP_R_16BF, HIP_R_32F};
  const long m = 4096, n = 16384, k = 1024;  // fc1 forward, column-major D[f x tokens]
  for (const Epi& ep : eps) {
    int total = 0;
    for (int ta = 0; ta < 2; ++ta)
      for (int tb = 0; tb < 2; ++tb)
        for (int ai = 0; ai < (ep.aux ? 3 : 1); ++ai)
          for (int bi = 0; bi < (ep.bias ? 2 : 1); ++bi) {
            hipblasLtMatmulDesc_t d;
            hipblasLtMatmulDescCreate(&d, HIPBLAS_COMPUTE_32F, HIP_R_32F);
            hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_TRANSA, &ops[ta], sizeof(ops[ta]));
            hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_TRANSB, &ops[tb], sizeof(ops[tb]));
            hipblasLtEpilogue_t e = ep.e;
            hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e));
            if (ep.bias)
              hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bias_types[bi],
                                              sizeof(hipDataType));
            if (ep.aux) {
              if (aux_types[ai] >= 0) {
                hipDataType at = (hipDataType)aux_types[ai];
                hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at, sizeof(at));
              }
              int64_t ld = m;
              hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld));
            }
            hipblasLtMatrixLayout_t la, lb, lc;
            if (ops[ta] == HIPBLAS_OP_N) hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, m, k, m);
            else hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, k, m, k);
            if (ops[tb] == HIPBLAS_OP_N) hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, k, n, k);
            else hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, n, k, n);
            hipblasLtMatrixLayoutCreate(&lc, HIP_R_16BF, m, n, m);
            hipblasLtMatmulPreference_t pref;
            hipblasLtMatmulPreferenceCreate(&pref);
            size_t ws = 64 << 20;
            hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
            hipblasLtMatmulHeuristicResult_t res[8];
            int cnt = 0;
            hipblasStatus_t s = hipblasLtMatmulAlgoGetHeuristic(h, d, la, lb, lc, lc, pref, 8, res, &cnt);
            if (s != HIPBLAS_STATUS_SUCCESS) cnt = 0;
            total += cnt;
            if (cnt > 0)
              printf("%-14s op%s%s aux=%-4s bias=%-4s : %d solutions\n", ep.name, opn[ta], opn[tb],
                     !ep.aux ? "-" : (ai == 0 ? "dflt" : (ai == 1 ? "bf16" : "f32")),
                     !ep.bias ? "-" : (bi == 0 ? "bf16" : "f32"), cnt);
            hipblasLtMatmulPreferenceDestroy(pref);
            hipblasLtMatrixLayoutDestroy(la);
            hipblasLtMatrixLayoutDestroy(lb);
            hipblasLtMatrixLayoutDestroy(lc);
            hipblasLtMatmulDescDestroy(d);
          }
    printf("== %-14s total %d\n", ep.name, total);
  }
  hipblasLtDestroy(h);
  return 0;
}
