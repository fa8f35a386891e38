// Reproducer for the gemm_pk packed-FP32 epilogue fault (tools/pk_diag.py): the instruction sequence
// hipcc 7.2 emitted for element 0 of the last accumulator block of gemm_pk<f16, 64x64> with packed-FP32
// VALU ops enabled, copied register for register (renamed into a clobbered range), run over every lane
// of many waves.  VARIANT selects s_nop padding: 0 = as emitted, 1 = s_nop 1 after v_pk_mov_b32,
// 2 = s_nop 1 after v_mov_b32 (before v_pk_add_f32), 3 = v_pk_mov_b32 replaced by two v_mov_b32.
// Optionally a second wave per SIMD runs MFMAs meanwhile (busy = 1).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

#define SEQ_HEAD                                                   \
  "v_mov_b32 v42, %2\n\tv_mov_b32 v43, %3\n\t"                     \
  "v_mov_b32 v50, %4\n\tv_mov_b32 v51, %5\n\t"                     \
  "v_mov_b32 v52, %6\n\tv_mov_b32 v53, %7\n\t"                     \
  "v_mov_b32 v62, 0\n\tv_mov_b32 v63, 0\n\tv_mov_b32 v44, 0\n\tv_mov_b32 v45, 0\n\t" \
  "s_nop 7\n\ts_nop 7\n\t"                                        \
  "v_add_f32_e32 v44, v51, v53\n\t"
#define SEQ_TAIL "s_nop 7\n\ts_nop 7\n\tv_mov_b32 %0, v44\n\tv_mov_b32 %1, v45\n\t"


#define IN6 "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5])
#define CLOB "v0", "v1", "v42", "v43", "v44", "v45", "v50", "v51", "v52", "v53", "v62", "v63", "s90", "s91", "s92", "s93"
#define PKMOV_GROUP(PAD1, PAD2)                                              \
  asm volatile(SEQ_HEAD "v_pk_mov_b32 v[62:63], v[42:43], v[50:51] op_sel:[1,0]\n\t" PAD1 \
               "v_mov_b32_e32 v45, v52\n\t" PAD2 "v_pk_add_f32 v[44:45], v[62:63], v[44:45]\n\t" SEQ_TAIL \
               : "=v"(o0), "=v"(o1) : IN6 : CLOB)
// consumer: v45 = v52 * v53 (VALU write), then the op_sel packed add; result lo = v42 + v45
#define OPSEL_GROUP(MID, OPS)                                                \
  asm volatile(SEQ_HEAD "v_mul_f32_e32 v45, v52, v53\n\t" MID                 \
               "v_pk_add_f32 v[0:1], v[42:43], v[44:45] " OPS "\n\t"       \
               "v_ashrrev_i32_e32 v1, 31, v50\n\t"                            \
               "s_nop 7\n\ts_nop 7\n\tv_mov_b32 %0, v0\n\tv_mov_b32 %1, v45\n\t" \
               : "=v"(o0), "=v"(o1) : IN6 : CLOB)
#define SALU3 "s_or_b64 s[90:91], exec, 0\n\ts_and_saveexec_b64 s[92:93], exec\n\ts_or_b64 exec, exec, s[92:93]\n\t"

template <int VARIANT>
__global__ void seq(const float* in, float* out, int busy_iters) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const float* p = in + 6 * gid;
  if (busy_iters > 0 && (threadIdx.x >> 6) & 1) {       // odd waves: MFMA load on the SIMD
    f32x4 acc = {0, 0, 0, 0};
    f16x8 a = {(_Float16)p[0], (_Float16)p[1], 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < busy_iters; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, a, acc, 0, 0, 0);
    out[2 * gid] = acc[0];
    out[2 * gid + 1] = acc[1];
    return;
  }
  float o0, o1;
  if constexpr (VARIANT == 0) PKMOV_GROUP("", "");
  else if constexpr (VARIANT == 1) PKMOV_GROUP("s_nop 1\n\t", "");
  else if constexpr (VARIANT == 2) PKMOV_GROUP("", "s_nop 1\n\t");
  else if constexpr (VARIANT == 3)
    asm volatile(SEQ_HEAD "v_mov_b32 v62, v43\n\tv_mov_b32 v63, v50\n\tv_mov_b32_e32 v45, v52\n\t"
                 "v_pk_add_f32 v[44:45], v[62:63], v[44:45]\n\t" SEQ_TAIL : "=v"(o0), "=v"(o1) : IN6 : CLOB);
  else if constexpr (VARIANT == 4) OPSEL_GROUP(SALU3, "op_sel:[0,1] op_sel_hi:[1,0]");
  else if constexpr (VARIANT == 5) OPSEL_GROUP("", "op_sel:[0,1] op_sel_hi:[1,0]");
  else if constexpr (VARIANT == 6) OPSEL_GROUP("s_nop 1\n\t", "op_sel:[0,1] op_sel_hi:[1,0]");
  else OPSEL_GROUP(SALU3, "");
  out[2 * gid] = o0;
  out[2 * gid + 1] = o1;
}

template <int V>
static void launch(const float* d_in, float* d_out, int blocks, int threads, int busy) {
  seq<V><<<blocks, threads>>>(d_in, d_out, busy * 64);
}

int main(int argc, char** argv) {
  const int blocks = 4096, threads = 256, n = blocks * threads, reps = argc > 1 ? atoi(argv[1]) : 20;
  float *h_in = (float*)malloc(6 * n * 4), *h_out = (float*)malloc(2 * n * 4);
  for (int i = 0; i < 6 * n; ++i) h_in[i] = 1.0f + (float)((i * 2654435761u) % 1000) / 7.0f;
  float *d_in, *d_out;
  (void)hipMalloc(&d_in, 6 * n * 4);
  (void)hipMalloc(&d_out, 2 * n * 4);
  (void)hipMemcpy(d_in, h_in, 6 * n * 4, hipMemcpyHostToDevice);
  void (*fns[8])(const float*, float*, int, int, int) = {launch<0>, launch<1>, launch<2>, launch<3>,
                                                         launch<4>, launch<5>, launch<6>, launch<7>};
  for (int busy = 0; busy < 2; ++busy)
    for (int v = 0; v < 8; ++v) {
      long bad = 0, bad4863 = 0, checked = 0;
      for (int r = 0; r < reps; ++r) {
        (void)hipMemset(d_out, 0xff, 2 * n * 4);
        fns[v](d_in, d_out, blocks, threads, busy);
        (void)hipMemcpy(h_out, d_out, 2 * n * 4, hipMemcpyDeviceToHost);
        for (int g = 0; g < n; ++g) {
          if (busy && ((g % threads) >> 6) & 1) continue;
          const float* p = h_in + 6 * g;
          float e0, e1;
          if (v < 4) { e0 = p[1] + (p[3] + p[5]); e1 = p[2] + p[4]; }
          else if (v < 7) { e1 = p[4] * p[5]; e0 = p[0] + e1; }     // lo = v42 + v45 (op_sel)
          else { e1 = p[4] * p[5]; e0 = p[0] + (p[3] + p[5]); }      // lo = v42 + v44, no op_sel
          ++checked;
          if (h_out[2 * g] != e0 || h_out[2 * g + 1] != e1) {
            ++bad;
            if ((g & 63) >= 48) ++bad4863;
          }
        }
      }
      printf("busy=%d variant=%d: %ld bad of %ld lane results (%ld in lanes 48-63)\n", busy, v, bad, checked, bad4863);
      fflush(stdout);
    }
  return 0;
}
