// f16 instantiations of the persistent GEMM (gemm_pk.hip)
#define SVK_PK_T f16
#include "gemm_pk.hip"
