// Host-side helpers shared by the GEMM / convolution entry points (mg_gemm.hip, mg_mx8.hip).
#pragma once
#include "mg_gemm.h"

namespace mg {

template <typename TO>
Epi<TO> make_epi(void* C, int64_t ldc, const mg_epilogue* e) {
  Epi<TO> ep;
  ep.C = reinterpret_cast<TO*>(C);
  ep.ldc = ldc;
  ep.gstride_c = 0;
  ep.alpha = e ? e->alpha : 1.f;
  ep.bias = e ? e->bias : nullptr;
  ep.gstride_bias = 0;
  ep.scale = e ? e->scale : nullptr;
  ep.scale_shift = e ? e->scale_shift : 0;
  ep.scale_ld = e ? e->scale_ld : 0;
  ep.rowscale = e ? e->rowscale : nullptr;
  ep.act = e ? e->act : 0;
  ep.aux = e ? reinterpret_cast<const TO*>(e->aux) : nullptr;
  ep.ld_aux = e ? e->ld_aux : 0;
  ep.resid = e ? reinterpret_cast<const TO*>(e->resid) : nullptr;
  ep.ld_res = e ? e->ld_res : 0;
  ep.accumulate = e ? e->accumulate : 0;
  ep.atomic = e ? e->atomic : 0;
  ep.remap_lgcin = e ? e->remap_lgcin : 0;
  ep.remap_taps = e ? e->remap_taps : 0;
  ep.addvec = e ? e->addvec : nullptr;
  ep.add_shift = e ? e->add_shift : 0;
  ep.add_ld = e ? e->add_ld : 0;
  ep.rm_mode = 0;
  ep.rm_Mc = 1;
  ep.rm_lgOW = ep.rm_lgOHW = 0;
  ep.Cpre = e ? reinterpret_cast<TO*>(e->out_pre) : nullptr;
  ep.ldc_pre = e ? e->ld_pre : 0;
  ep.zstride = 0;
  ep.zi = 0;
  ep.vec_ok = 0;
  ep.g = 0;
  return ep;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
// Operands are fetched through buffer descriptors with 32-bit byte offsets (mg_gemm.h): every operand's
// byte extent must stay below 2 GiB, or loads past it would silently return zeros.
inline bool under2g(int64_t elems, int dtype) {
  return elems >= 0 && elems * (dtype == MG_F32 ? 4 : 2) < (int64_t)0x7fffff00;
}
inline int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}
inline bool pow2(int v) { return v > 0 && (v & (v - 1)) == 0; }
inline int kwinv(int KW) { return 65536 / KW + 1; }  // exact tap / KW for tap < 64

}  // namespace mg
