// Trace-time specialisation of site-group kernels (hiprtc, gfx950).
//
// A traced model yields site groups whose structure -- families, which role of which site reads
// which operand, whether an operand varies per particle and/or per element, masks, and where each
// partial derivative goes -- is fixed for the life of a training loop. The precompiled generic
// kernels in sites.hip interpret that structure at run time, which puts uniform branches around
// every load (hipcc then waits vmcnt(0) per element) and runtime-indexed register selects into the
// element loop. Here the structure becomes compile-time: the generator below emits straight-line
// HIP for exactly one group signature (every load unconditional, every gradient target a named
// register, per-particle and constant roles hoisted by the compiler), hiprtc compiles it once per
// signature and the code object is cached for the process. Pointers, strides, constants and scales
// stay kernel arguments (the same mi_group block), so one compiled kernel serves every step.
//
// The family math is the same device code the precompiled kernels use (device_math.hpp, embedded
// verbatim), so both paths compute identical values.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "jit.hpp"

namespace {

const char kHeaderText[] =
#include "embedded_header.inc"
    ;
const char kMathText[] =
#include "embedded_math.inc"
    ;
const char kStddefStub[] =
    "#pragma once\ntypedef __SIZE_TYPE__ size_t;\ntypedef __PTRDIFF_TYPE__ ptrdiff_t;\n";

enum Kind { kConst = 0, kBroadcast = 1, kShared = 2, kParticle = 3, kDense = 4 };

// LDS table of a program's per-particle draw (mi_group.pdraw): sites.hip kPdrawMax particles
constexpr int kPdrawTable = 1024;

Kind kind_of(int64_t sk, int64_t si) {
  if (sk == 0 && si == 0) return kBroadcast;
  if (sk == 0) return kShared;
  if (si == 0) return kParticle;
  return kDense;
}

const char* eval_fn(int family) {
  switch (family) {
    case MI_NORMAL: return "eval_normal";
    case MI_BERNOULLI_LOGITS: return "eval_bernoulli_logits";
    case MI_BERNOULLI_PROBS: return "eval_bernoulli_probs";
    case MI_GAMMA: return "eval_gamma";
    case MI_POISSON: return "eval_poisson";
    case MI_INVERSE_GAMMA: return "eval_inverse_gamma";
    default: return "eval_beta";
  }
}

// Families whose density has no second parameter role (their eval_* take (r0, value)).
bool one_param(int family) {
  return family == MI_BERNOULLI_LOGITS || family == MI_BERNOULLI_PROBS || family == MI_POISSON;
}

bool role_used(int family, int q) { return !(one_param(family) && q == 1); }

// Families with packed-pair evaluations (device_math.hpp eval_*2).
bool packed_family(int family) { return family == MI_NORMAL || family == MI_BERNOULLI_LOGITS; }

// Whether the fused-draw loop of `g` runs on element pairs (PlanInfo.packed, when every site has a
// packed form and the lane's elements pair up).
bool use_packed(const mi_group& g, const PlanInfo& plan) {
  if (!plan.packed || plan.elems % 2 != 0) return false;
  for (int s = 0; s < g.num_sites; ++s)
    if (!packed_family(g.sites[s].family)) return false;
  return true;
}

// Everything about a group that changes the generated code.
struct Signature {
  std::string text;
};

// Per-element values are arrays indexed by `e` (ROW: the lane's E elements of a row segment;
// COL: E unrolled element iterations); per-particle values are scalars.
std::string operand_var(const mi_group& g, int o) {
  switch (kind_of(g.operands[o].stride_k, g.operands[o].stride_i)) {
    case kBroadcast: return "b" + std::to_string(o);
    case kShared: return "s" + std::to_string(o) + "[e]";
    case kParticle: return "p" + std::to_string(o);
    default: return "d" + std::to_string(o) + "[e]";
  }
}

std::string mask_var(const mi_site& st, int s) {
  switch (kind_of(st.mask_stride_k, st.mask_stride_i)) {
    case kBroadcast: return "m" + std::to_string(s);
    case kShared: return "m" + std::to_string(s) + "[e]";
    case kParticle: return "mp" + std::to_string(s);
    default: return "md" + std::to_string(s) + "[e]";
  }
}

std::string mask_kind_tag(const mi_site& st) {
  if (st.mask == nullptr) return "-";
  return std::to_string((int)kind_of(st.mask_stride_k, st.mask_stride_i));
}

// MININF_AMD_DRAW_PAIRS=1: the fused-draw accumulator loop takes two particles per iteration as
// two independent Philox -> Box-Muller -> density chains (opt-in: measured slower on MI355X, round
// 6 -- C5's program 153.4-154.0 us against 151.7-152.5 with one chain, profiles/r06_c5_ab.json).
// Read per compile; part of the signature.
bool draw_pairs() {
  const char* v = std::getenv("MININF_AMD_DRAW_PAIRS");
  return v != nullptr && std::atoi(v) != 0;
}

Signature signature(const mi_group& g, const PlanInfo& plan) {
  std::ostringstream s;
  s << (plan.row ? "R" : "C") << plan.elems << "/" << plan.kw << (plan.combined ? "c" : "s")
    << (plan.block_rows ? "B" : "") << (use_packed(g, plan) ? "P" : "") << "|"
    << g.num_operands << ":";
  for (int o = 0; o < g.num_operands; ++o) {
    const mi_operand& op = g.operands[o];
    s << (int)kind_of(op.stride_k, op.stride_i) << (g.compute_grads ? op.grad_mode : 0)
      << (op.grad_mode == MI_GRAD_PARTICLE ? op.slot : 0) << (op.stride_i == 1 ? "u" : "")
      << (op.grad_stride_i == 1 ? "v" : "") << ",";
  }
  s << "|" << g.num_sites << ":";
  for (int i = 0; i < g.num_sites; ++i) {
    const mi_site& st = g.sites[i];
    s << st.family << "(" << st.operand[0] << "," << st.operand[1] << "," << st.operand[2] << ","
      << mask_kind_tag(st) << (st.mask_stride_i == 1 ? "u" : "") << ")";
  }
  s << "|" << g.num_slots << "|" << g.compute_grads
    << (plan.row && g.N < 64L * plan.elems ? "|small" : "") << "|draw" << g.draw.operand
    << (g.draw.loc_stride == 0 ? "b" : "") << (g.draw.scale_stride == 0 ? "b" : "")
    << (g.draw.scale_exp != nullptr ? "x" : "")
    << (g.prior.present != 0 ? "|prior" + std::to_string(g.prior.family) : "")
    << (g.pdraw.operand != 0 ? "|pdraw" + std::to_string(g.pdraw.operand) : "");
  if (g.draw.operand != 0) s << "|pairs" << draw_pairs();
  return Signature{s.str()};
}

// ---- source generation ----------------------------------------------------------------------

void emit_site_eval(std::ostringstream& o, const mi_group& g, int s, const std::string& valid,
                    const char* in) {
  const mi_site& st = g.sites[s];
  std::string r[3];
  for (int q = 0; q < 3; ++q) {
    if (!role_used(st.family, q)) r[q] = "0.0f";
    else if (st.operand[q] < 0) r[q] = "c" + std::to_string(s) + "_" + std::to_string(q);
    else r[q] = operand_var(g, st.operand[q]);
  }
  o << in << "{\n" << in << "  mi::Elem el;\n";
  if (one_param(st.family))
    o << in << "  mi::" << eval_fn(st.family) << "(" << r[0] << ", " << r[2] << ", el);\n";
  else
    o << in << "  mi::" << eval_fn(st.family) << "(" << r[0] << ", " << r[1] << ", " << r[2]
      << ", el);\n";
  std::string obs = valid;
  if (st.mask != nullptr) obs = "(" + obs + " && " + mask_var(st, s) + ")";
  o << in << "  const bool obs = " << obs << ";\n";
  o << in << "  lp" << s << " += obs ? el.lp : 0.0f;\n";
  // lane-mask booleans (scalar ORs of the compare results), turned into flag bits once at the end
  o << in << "  pb" << s << " |= el.param_bad;\n" << in << "  sb" << s
    << " |= obs && el.support_bad;\n";
  if (g.compute_grads) {
    bool any = false;
    for (int q = 0; q < 3; ++q) {
      const int op = st.operand[q];
      if (op >= 0 && role_used(st.family, q) && g.operands[op].grad_mode != MI_GRAD_NONE) any = true;
    }
    if (any) o << in << "  const float w = obs ? scale" << s << " : 0.0f;\n";
    for (int q = 0; q < 3; ++q) {
      const int op = st.operand[q];
      if (op < 0 || !role_used(st.family, q)) continue;
      if (g.operands[op].grad_mode == MI_GRAD_DENSE)
        o << in << "  g" << op << "[e] = fmaf(w, el.d[" << q << "], g" << op << "[e]);\n";
      else if (g.operands[op].grad_mode == MI_GRAD_PARTICLE)
        o << in << "  sl" << g.operands[op].slot << " = fmaf(w, el.d[" << q << "], sl"
          << g.operands[op].slot << ");\n";
    }
  }
  o << in << "}\n";
}

// Element `comp` (0 or 1) of pair h of a per-element expression ("s2[e]" -> "s2[2 * h + 1]").
std::string at_pair(std::string x, int comp) {
  const std::string to = comp ? "[2 * h + 1]" : "[2 * h]";
  for (size_t i = x.find("[e]"); i != std::string::npos; i = x.find("[e]", i + to.size()))
    x.replace(i, 3, to);
  return x;
}

// A role's value for pair h as an f2: per-element operands pair up, the rest are splatted.
std::string pair_role(const std::string& x) {
  if (x.find("[e]") == std::string::npos) return "mi::splat2(" + x + ")";
  return "mi::f2{" + at_pair(x, 0) + ", " + at_pair(x, 1) + "}";
}

// emit_site_eval for element pair h (elements 2h, 2h + 1): the arithmetic of each element is that
// of the scalar form, the log-probability and slot sums keep the scalar order (element 2h, then
// 2h + 1), dense gradients accumulate per element as f2.
void emit_site_eval2(std::ostringstream& o, const mi_group& g, int s, const std::string& valid,
                     const char* in) {
  const mi_site& st = g.sites[s];
  std::string r[3];
  for (int q = 0; q < 3; ++q) {
    if (!role_used(st.family, q)) r[q] = "0.0f";
    else if (st.operand[q] < 0) r[q] = "c" + std::to_string(s) + "_" + std::to_string(q);
    else r[q] = operand_var(g, st.operand[q]);
  }
  o << in << "{\n" << in << "  mi::Elem2 el;\n";
  if (one_param(st.family))
    o << in << "  mi::" << eval_fn(st.family) << "2(" << pair_role(r[0]) << ", " << pair_role(r[2])
      << ", el);\n";
  else
    o << in << "  mi::" << eval_fn(st.family) << "2(" << pair_role(r[0]) << ", " << pair_role(r[1])
      << ", " << pair_role(r[2]) << ", el);\n";
  std::string obs = valid;
  if (st.mask != nullptr) obs = "(" + obs + " && " + mask_var(st, s) + ")";
  o << in << "  const bool obs0 = " << at_pair(obs, 0) << ", obs1 = " << at_pair(obs, 1) << ";\n";
  o << in << "  lp" << s << " += obs0 ? el.lp.x : 0.0f;\n";
  o << in << "  lp" << s << " += obs1 ? el.lp.y : 0.0f;\n";
  o << in << "  pb" << s << " |= el.param_bad;\n" << in << "  sb" << s
    << " |= (obs0 & el.support_bad[0]) | (obs1 & el.support_bad[1]);\n";
  if (g.compute_grads) {
    bool any = false;
    for (int q = 0; q < 3; ++q) {
      const int op = st.operand[q];
      if (op >= 0 && role_used(st.family, q) && g.operands[op].grad_mode != MI_GRAD_NONE) any = true;
    }
    if (any)
      o << in << "  const mi::f2 w = mi::f2{obs0 ? scale" << s << " : 0.0f, obs1 ? scale" << s
        << " : 0.0f};\n";
    for (int q = 0; q < 3; ++q) {
      const int op = st.operand[q];
      if (op < 0 || !role_used(st.family, q)) continue;
      if (g.operands[op].grad_mode == MI_GRAD_DENSE)
        o << in << "  g" << op << "[h] = mi::fma2(w, el.d[" << q << "], g" << op << "[h]);\n";
      else if (g.operands[op].grad_mode == MI_GRAD_PARTICLE) {
        const std::string sl = "sl" + std::to_string(g.operands[op].slot);
        o << in << "  " << sl << " = fmaf(w.x, el.d[" << q << "].x, " << sl << ");\n";
        o << in << "  " << sl << " = fmaf(w.y, el.d[" << q << "].y, " << sl << ");\n";
      }
    }
  }
  o << in << "}\n";
}


// ---- accumulator forms (fused-draw packed loop) ----------------------------------------------
// In the fused-draw row loop every site's per-element log density enters only the row's sum, so
// instead of evaluating the full density per element (eval_*2: every role's derivative, the
// constant terms, a select and an add per element) the loop accumulates what the density is
// affine in, per element pair:
//   Normal(loc, sigma) with sigma constant or per-particle: t = obs ? v - loc : 0, Sum t^2 (and
//     Sum t when a per-particle role takes a slot gradient); per element the gradients are
//     +-sigma^-2 t, one packed FMA into the dense target. The row's log density is
//     -sigma^-2 / 2 Sum t^2 + n_obs (-log sigma - log sqrt(2 pi)), n_obs per lane being
//     loop-invariant (the masks and the lane's validity do not change with the particle).
//   Bernoulli(logits l): lp = v l - max(l, 0) - log(1 + exp(-|l|)) on the hardware exp / log / rcp,
//     Sum obs ? lp : 0; d/dl = v - sigmoid(l).
// Same formulas as device_math.hpp's eval_normal2 / eval_bernoulli_logits2 up to rounding order
// (the constant terms are added once per row, not per element; log1p(t) is log(fl(1 + t)) without
// eval_bernoulli_logits2's first-order correction for the rounding of 1 + t: an absolute error
// below 2^-24 per element, far inside the 1e-5 relative tolerance of every ELBO and gradient).
// The accumulator form applies when every site of the group qualifies (acc_form).
bool acc_site(const mi_group& g, int s, int draw) {
  const mi_site& st = g.sites[s];
  if (st.mask != nullptr && kind_of(st.mask_stride_k, st.mask_stride_i) != kShared) return false;
  auto op_kind = [&](int q) {
    const int o = st.operand[q];
    return o < 0 ? kConst : kind_of(g.operands[o].stride_k, g.operands[o].stride_i);
  };
  auto grad_of = [&](int q) {
    const int o = st.operand[q];
    return (o < 0 || !g.compute_grads) ? (int)MI_GRAD_NONE : (int)g.operands[o].grad_mode;
  };
  if (st.family == MI_NORMAL) {
    const Kind ks = op_kind(1);
    if (!(ks == kConst || ks == kParticle || ks == kBroadcast)) return false;
    if (st.operand[0] >= 0 && st.operand[0] == st.operand[2]) return false;
    for (int q = 0; q < 3; ++q)
      if (st.operand[q] >= 0 && (st.operand[q] == st.operand[1]) && q != 1) return false;
    if (grad_of(1) == MI_GRAD_DENSE) return false;
    return true;
  }
  if (st.family == MI_BERNOULLI_LOGITS) {
    if (grad_of(2) != MI_GRAD_NONE) return false;   // (a gradient w.r.t. the observed value)
    return true;
  }
  return false;
}

bool acc_form(const mi_group& g, int draw) {
  if (std::getenv("MININF_AMD_ACC_FORM") != nullptr && std::atoi(std::getenv("MININF_AMD_ACC_FORM")) == 0)
    return false;
  for (int s = 0; s < g.num_sites; ++s)
    if (!acc_site(g, s, draw)) return false;
  return true;
}

std::string generate(const mi_group& g, const PlanInfo& plan) {
  const bool row = plan.row;
  const int E = plan.elems;
  const std::string Es = std::to_string(E);
  const int nsite_values = plan.combined ? 1 : g.num_sites;
  const int nv = nsite_values + (g.compute_grads ? g.num_slots : 0);
  const bool packed = use_packed(g, plan);
  // a folded prior site (mi_prior): evaluated at the block-row flush (combined values only)
  const bool prior = g.prior.present != 0 && row && plan.block_rows && plan.combined;
  const int pdraw = g.pdraw.operand - 1;   // a per-particle draw made by the program (or -1)
  std::ostringstream o;
  auto is = [&](int op, Kind k) { return kind_of(g.operands[op].stride_k, g.operands[op].stride_i) == k; };
  auto mask_is = [&](int s, Kind k) {
    return g.sites[s].mask != nullptr && kind_of(g.sites[s].mask_stride_k, g.sites[s].mask_stride_i) == k;
  };
  auto dense_grad = [&](int op) { return g.compute_grads && g.operands[op].grad_mode == MI_GRAD_DENSE; };

  const int draw = g.draw.operand - 1;
  o << "#include \"device_math.hpp\"\n";
  o << "extern \"C\" __global__ __launch_bounds__(256) ";
  o << "void mi_site_program(const mi_group G, "
       "float* __restrict__ part, long nseg, long arg, unsigned* __restrict__ flags) {\n";
  // the descriptor's lines into L2 with one vector load (device_math.hpp kernarg_prefetch): the
  // program's draw and prior prologue reads it in dependent chains
  o << "  mi::kernarg_prefetch<(int)sizeof(mi_group)>();\n";
  o << "  const unsigned long long span_t0 = mi::span_begin(G.stamps);\n";
  o << "  const int lane = threadIdx.x & 63;\n";
  o << "  const long seg = (long)blockIdx.x * 4 + (threadIdx.x >> 6);\n";
  o << "  const long K = G.K, N = G.N;\n";
  // LDS of the row loops' particle sums: nv tiles of [tile_rows][65] floats per wave
  const int tile_rows = nv <= 2 ? 16 : 8;
  if (row)
    o << "  __shared__ float red[" << 4 * nv * tile_rows * 65 << "];\n"
      << "  float* const tile = red + (threadIdx.x >> 6) * " << nv * tile_rows * 65 << ";\n";
  for (int s = 0; s < g.num_sites; ++s) {
    o << "  bool pb" << s << " = false, sb" << s << " = false;\n";
    o << "  const float scale" << s << " = (float)G.sites[" << s << "].scale;\n";
    for (int q = 0; q < 3; ++q)
      if (g.sites[s].operand[q] < 0 && role_used(g.sites[s].family, q))
        o << "  const float c" << s << "_" << q << " = G.sites[" << s << "].constant[" << q << "];\n";
  }
  for (int op = 0; op < g.num_operands; ++op) {
    o << "  const float* __restrict__ x" << op << " = G.operands[" << op << "].data;\n";
    o << "  const long sk" << op << " = G.operands[" << op << "].stride_k, si" << op
      << " = G.operands[" << op << "].stride_i;\n";
    if (dense_grad(op)) {
      o << "  float* __restrict__ gx" << op << " = G.operands[" << op << "].grad;\n";
      o << "  const long gsk" << op << " = G.operands[" << op << "].grad_stride_k, gsi" << op
        << " = G.operands[" << op << "].grad_stride_i;\n";
    }
    if (is(op, kBroadcast)) o << "  const float b" << op << " = x" << op << "[0];\n";
  }
  for (int s = 0; s < g.num_sites; ++s) {
    if (g.sites[s].mask == nullptr) continue;
    o << "  const unsigned char* __restrict__ mk" << s << " = G.sites[" << s << "].mask;\n";
    o << "  const long msk" << s << " = G.sites[" << s << "].mask_stride_k, msi" << s
      << " = G.sites[" << s << "].mask_stride_i;\n";
    if (mask_is(s, kBroadcast)) o << "  const bool m" << s << " = mk" << s << "[0] != 0;\n";
  }
  auto value_expr = [&](int v) -> std::string {
    if (v < nsite_values) {
      if (!plan.combined) return "lp" + std::to_string(v);
      std::string e;
      for (int s = 0; s < g.num_sites; ++s)
        e += (s ? " + " : "") + std::string("scale") + std::to_string(s) + " * lp" + std::to_string(s);
      return "(" + e + ")";
    }
    return "sl" + std::to_string(v - nsite_values);
  };
  auto zero_accumulators = [&](const char* in) {
    for (int s = 0; s < g.num_sites; ++s) o << in << "float lp" << s << " = 0.0f;\n";
    if (g.compute_grads)
      for (int j = 0; j < g.num_slots; ++j) o << in << "float sl" << j << " = 0.0f;\n";
  };
  auto particle_loads = [&](const char* in, const char* kexpr) {
    for (int op = 0; op < g.num_operands; ++op)
      if (is(op, kParticle))
        o << in << "const float p" << op << " = x" << op << "[" << kexpr << " * sk" << op << "];\n";
    for (int s = 0; s < g.num_sites; ++s)
      if (mask_is(s, kParticle))
        o << in << "const bool mp" << s << " = mk" << s << "[" << kexpr << " * msk" << s << "] != 0;\n";
  };
  // Dense (particle x element) loads of one row / chunk into arrays `prefix`<op>[e].
  auto dense_loads = [&](const char* in, const char* prefix, const std::string& kexpr,
                         const char* iexpr) {
    for (int op = 0; op < g.num_operands; ++op)
      if (is(op, kDense))
        o << in << "#pragma unroll\n" << in << "for (int e = 0; e < " << Es << "; ++e) " << prefix
          << op << "[e] = x" << op << "[" << kexpr << " * sk" << op << " + " << iexpr << " * si"
          << op << "];\n";
    for (int s = 0; s < g.num_sites; ++s)
      if (mask_is(s, kDense))
        o << in << "#pragma unroll\n" << in << "for (int e = 0; e < " << Es << "; ++e) " << prefix
          << "m" << s << "[e] = mk" << s << "[" << kexpr << " * msk" << s << " + " << iexpr
          << " * msi" << s << "] != 0;\n";
  };
  auto compute_and_store = [&](const char* in, const std::string& valid, const char* kexpr,
                               const char* iexpr) {
    for (int op = 0; op < g.num_operands; ++op)
      if (dense_grad(op)) o << in << "float g" << op << "[" << Es << "];\n";
    o << in << "#pragma unroll\n" << in << "for (int e = 0; e < " << Es << "; ++e) {\n";
    const std::string inner = std::string(in) + "  ";
    for (int op = 0; op < g.num_operands; ++op)
      if (dense_grad(op)) o << inner << "g" << op << "[e] = 0.0f;\n";
    for (int s = 0; s < g.num_sites; ++s) emit_site_eval(o, g, s, valid, inner.c_str());
    o << in << "}\n";
    for (int op = 0; op < g.num_operands; ++op)
      if (dense_grad(op))
        o << in << "#pragma unroll\n" << in << "for (int e = 0; e < " << Es << "; ++e) if ("
          << valid << ") gx" << op << "[" << kexpr << " * gsk" << op << " + " << iexpr << " * gsi"
          << op << "] = G.grad_scale * g" << op << "[e];\n";
  };
  auto declare_dense = [&](const char* in, const char* prefix) {
    for (int op = 0; op < g.num_operands; ++op)
      if (is(op, kDense)) o << in << "float " << prefix << op << "[" << Es << "];\n";
    for (int s = 0; s < g.num_sites; ++s)
      if (mask_is(s, kDense)) o << in << "bool " << prefix << "m" << s << "[" << Es << "];\n";
  };

  // Per-particle sums over the wave's elements (the row loops): each particle's lane values go to
  // a [tile_rows][65] LDS tile of the wave, and every tile_rows particles the wave sums the rows
  // (mi::tile_row_sums: tile_rows columns per lane, then a shuffle tree over the row's lanes) --
  // about one LDS write, one LDS read and one add per particle and value, where a shuffle
  // reduction per particle costs six exchanges and six adds.
  // block_rows: the block's four waves combine their row sums in LDS (fixed wave order) and write
  // one partial row per block (gridDim.x rows) -- a quarter of the partials, short enough for the
  // ELBO forward's fused reduction; every wave then runs the loop (see emit_draw_loop).
  // write = false: the caller wrote the tile rows (the paired fused-draw loop)
  auto emit_particle_sums = [&](const char* in, bool block_rows, bool write = true) {
    if (write)
      for (int v = 0; v < nv; ++v)
        o << in << "tile[" << v * tile_rows * 65 << " + r * 65 + lane] = " << value_expr(v) << ";\n";
    o << in << "if (r == " << tile_rows - 1 << " || k + 1 == k_end) {\n";
    o << in << "  mi::wave_lds_sync();\n";
    if (!block_rows) {
      for (int v = 0; v < nv; ++v)
        o << in << "  { const float t = mi::tile_row_sums<" << tile_rows << ">(tile + "
          << v * tile_rows * 65 << ", lane);\n" << in << "    if (lane <= r) part[((long)" << v
          << " * nseg + seg) * K + (k - r) + lane] = t; }\n";
      o << in << "  mi::wave_lds_sync();\n";
    } else {
      for (int v = 0; v < nv; ++v)
        o << in << "  { const float t = mi::tile_row_sums<" << tile_rows << ">(tile + "
          << v * tile_rows * 65 << ", lane);\n" << in << "    if (lane < " << tile_rows
          << ") bsum[(" << v << " * 4 + (threadIdx.x >> 6)) * " << tile_rows << " + lane] = t; }\n";
      o << in << "  __syncthreads();\n";
      o << in << "  if (threadIdx.x < " << tile_rows << " && (int)threadIdx.x <= r) {\n";
      if (prior) {
        // the folded prior site (mi_prior) on site 0's per-particle parameter: its log density
        // and d/dparameter enter the particle's value and the parameter's slot once, from the
        // writer threads of block column 0 (the prior's scale equals site 0's)
        const int po = g.sites[0].operand[0];
        o << in << "    float pv = 0.0f, pd = 0.0f;\n";
        o << in << "    if (blockIdx.x == 0) {\n";
        if (po == pdraw)
          o << in << "      const float a = pdv[(k - r) + (long)threadIdx.x - k_begin];\n";
        else
          o << in << "      const float a = x" << po << "[((k - r) + (long)threadIdx.x) * sk" << po << "];\n";
        o << in << "      mi::Elem pe;\n";
        o << in << "      mi::" << (g.prior.family == MI_BETA ? "eval_beta" : g.prior.family == MI_NORMAL
                                    ? "eval_normal" : "eval_gamma")
          << "(G.prior.constant[0], G.prior.constant[1], a, pe);\n";
        o << in << "      pv = (float)G.prior.scale * pe.lp;\n";
        o << in << "      pd = (float)G.prior.scale * pe.d[2];\n";
        o << in << "      const unsigned pf = (pe.param_bad ? " << MI_FLAG_PARAM << "u : 0u) | (pe.support_bad ? "
          << MI_FLAG_SUPPORT << "u : 0u);\n";
        o << in << "      if (pf != 0u) atomicOr(G.prior.flags, pf);\n";
        o << in << "    }\n";
      }
      for (int v = 0; v < nv; ++v) {
        std::string extra;
        if (prior && v == 0) extra = " + pv";
        if (prior && g.compute_grads && v >= nsite_values &&
            g.operands[g.sites[0].operand[0]].grad_mode == MI_GRAD_PARTICLE &&
            v - nsite_values == g.operands[g.sites[0].operand[0]].slot)
          extra = " + pd";
        o << in << "    part[((long)" << v << " * gridDim.x + blockIdx.x) * K + (k - r) + threadIdx.x] = "
          << "((bsum[(" << v << " * 4) * " << tile_rows << " + threadIdx.x] + bsum[(" << v
          << " * 4 + 1) * " << tile_rows << " + threadIdx.x]) + bsum[(" << v << " * 4 + 2) * "
          << tile_rows << " + threadIdx.x]) + bsum[(" << v << " * 4 + 3) * " << tile_rows
          << " + threadIdx.x]" << extra << ";\n";
      }
      o << in << "  }\n";
      o << in << "  __syncthreads();\n";
    }
    o << in << "}\n";
  };

  // One copy of the row loop (see below). Element e of the lane: `ie` in the clamped copy.
  auto emit_row_loop = [&](bool full) {
    const std::string ie = full ? "(base + e * 64 + lane)" : "idx[e]";
    const std::string valid = "ok[e]";
    auto unit = [&](int op) { return full && g.operands[op].stride_i == 1; };
    auto unit_grad = [&](int op) { return full && g.operands[op].grad_stride_i == 1; };
    auto unit_mask = [&](int s) { return full && g.sites[s].mask_stride_i == 1; };
    const char* in = "      ";
    if (!full)
      o << in << "long idx[" << E << "]; bool ok[" << E << "];\n#pragma unroll\n" << in
        << "for (int e = 0; e < " << E << "; ++e) { const long i = base + e * 64 + lane; "
           "ok[e] = i < N; idx[e] = ok[e] ? i : N - 1; }\n";
    else
      o << in << "bool ok[" << E << "];\n#pragma unroll\n" << in << "for (int e = 0; e < " << E
        << "; ++e) ok[e] = e * 64 + lane >= shift;\n";
    for (int op = 0; op < g.num_operands; ++op)
      if (is(op, kShared)) {
        o << in << "float s" << op << "[" << E << "];\n";
        if (unit(op))
          o << in << "{ const float* __restrict__ r = x" << op << " + base + lane;\n#pragma unroll\n"
            << in << "for (int e = 0; e < " << E << "; ++e) s" << op << "[e] = r[e * 64]; }\n";
        else
          o << "#pragma unroll\n" << in << "for (int e = 0; e < " << E << "; ++e) s" << op
            << "[e] = x" << op << "[" << ie << " * si" << op << "];\n";
      }
    for (int s = 0; s < g.num_sites; ++s)
      if (mask_is(s, kShared)) {
        o << in << "bool m" << s << "[" << E << "];\n";
        if (unit_mask(s))
          o << in << "{ const unsigned char* __restrict__ r = mk" << s << " + base + lane;\n#pragma unroll\n"
            << in << "for (int e = 0; e < " << E << "; ++e) m" << s << "[e] = r[e * 64] != 0; }\n";
        else
          o << "#pragma unroll\n" << in << "for (int e = 0; e < " << E << "; ++e) m" << s
            << "[e] = mk" << s << "[" << ie << " * msi" << s << "] != 0;\n";
      }
    // Dense (particle x element) loads of row `kexpr` into `prefix`<op>[e].
    auto row_loads = [&](const char* ind, const char* prefix, const std::string& kexpr) {
      for (int op = 0; op < g.num_operands; ++op)
        if (is(op, kDense)) {
          if (unit(op))
            o << ind << "{ const float* __restrict__ r = x" << op << " + " << kexpr << " * sk" << op
              << " + base + lane;\n#pragma unroll\n" << ind << "for (int e = 0; e < " << E << "; ++e) "
              << prefix << op << "[e] = r[e * 64]; }\n";
          else
            o << "#pragma unroll\n" << ind << "for (int e = 0; e < " << E << "; ++e) " << prefix << op
              << "[e] = x" << op << "[" << kexpr << " * sk" << op << " + " << ie << " * si" << op << "];\n";
        }
      for (int s = 0; s < g.num_sites; ++s)
        if (mask_is(s, kDense))
          o << "#pragma unroll\n" << ind << "for (int e = 0; e < " << E << "; ++e) " << prefix << "m" << s
            << "[e] = mk" << s << "[" << kexpr << " * msk" << s << " + " << ie << " * msi" << s
            << "] != 0;\n";
    };
    // software pipeline: the next row's dense values are in flight while this row computes
    declare_dense(in, "n");
    o << in << "if (k_begin < k_end) {\n";
    row_loads("        ", "n", "k_begin");
    o << in << "}\n";
    o << in << "for (long k = k_begin; k < k_end; ++k) {\n";
    o << in << "  const int r = (int)((k - k_begin) & " << tile_rows - 1 << ");\n";
    declare_dense("        ", "d");
    for (int op = 0; op < g.num_operands; ++op)
      if (is(op, kDense))
        o << "#pragma unroll\n" << in << "  for (int e = 0; e < " << E << "; ++e) d" << op << "[e] = n"
          << op << "[e];\n";
    for (int s = 0; s < g.num_sites; ++s)
      if (mask_is(s, kDense))
        o << "#pragma unroll\n" << in << "  for (int e = 0; e < " << E << "; ++e) dm" << s << "[e] = nm"
          << s << "[e];\n";
    o << in << "  if (k + 1 < k_end) {\n";
    row_loads("          ", "n", "(k + 1)");
    o << in << "  }\n";
    particle_loads("        ", "k");
    zero_accumulators("        ");
    const char* in2 = "        ";
    for (int op = 0; op < g.num_operands; ++op)
      if (dense_grad(op)) o << in2 << "float g" << op << "[" << E << "];\n";
    o << in2 << "#pragma unroll\n" << in2 << "for (int e = 0; e < " << E << "; ++e) {\n";
    const std::string inner = std::string(in2) + "  ";
    for (int op = 0; op < g.num_operands; ++op)
      if (dense_grad(op)) o << inner << "g" << op << "[e] = 0.0f;\n";
    for (int s = 0; s < g.num_sites; ++s) emit_site_eval(o, g, s, valid, inner.c_str());
    o << in2 << "}\n";
    for (int op = 0; op < g.num_operands; ++op)
      if (dense_grad(op)) {
        if (unit_grad(op))
          o << in2 << "{ float* __restrict__ r = gx" << op << " + k * gsk" << op
            << " + base + lane;\n#pragma unroll\n" << in2 << "for (int e = 0; e < " << E
            << "; ++e) if (ok[e]) r[e * 64] = G.grad_scale * g" << op << "[e]; }\n";
        else
          o << in2 << "#pragma unroll\n" << in2 << "for (int e = 0; e < " << E << "; ++e) if (" << valid
            << ") gx" << op << "[k * gsk" << op << " + " << ie << " * gsi" << op
            << "] = G.grad_scale * g" << op << "[e];\n";
      }
    emit_particle_sums(in2, false);
    o << in << "}\n";
  };


  // ---- accumulator forms (acc_form): per-site code of the fused-draw packed loop -------------
  auto site_str = [&](int s) { return std::to_string(s); };
  auto role_expr = [&](int s, int q) -> std::string {
    const mi_site& st = g.sites[s];
    if (st.operand[q] < 0) return "c" + site_str(s) + "_" + std::to_string(q);
    return operand_var(g, st.operand[q]);
  };
  auto site_obs = [&](int s, const std::string& valid) -> std::string {
    const mi_site& st = g.sites[s];
    std::string obs = valid;
    if (st.mask != nullptr) obs = (valid == "true") ? mask_var(st, s) : "(" + valid + " && " + mask_var(st, s) + ")";
    return obs;
  };
  auto role_grad = [&](int s, int q) -> int {
    const int op = g.sites[s].operand[q];
    if (op < 0 || !g.compute_grads || !role_used(g.sites[s].family, q)) return MI_GRAD_NONE;
    return g.operands[op].grad_mode;
  };
  auto normal_scale_const = [&](int s) { return g.sites[s].operand[1] < 0; };
  auto normal_needs_q1 = [&](int s) {
    return role_grad(s, 0) == MI_GRAD_PARTICLE || role_grad(s, 2) == MI_GRAD_PARTICLE;
  };
  // loop-invariant per lane: observed-element counts, constant-scale factors, the constant
  // parameters' checks
  auto emit_acc_prologue = [&](const std::string& valid) {
    const char* in = "    ";
    for (int st = 0; st < g.num_sites; ++st) {
      const std::string S = site_str(st);
      o << in << "float cn" << S << " = 0.0f;\n#pragma unroll\n" << in << "for (int e = 0; e < " << E
        << "; ++e) cn" << S << " += (" << site_obs(st, valid) << ") ? 1.0f : 0.0f;\n";
      if (g.sites[st].family == MI_NORMAL && normal_scale_const(st)) {
        const std::string sig = role_expr(st, 1);
        o << in << "const float iv" << S << " = mi::rcp(" << sig << "), iq" << S << " = iv" << S << " * iv" << S
          << ";\n" << in << "const float lc" << S << " = -(logf(" << sig << ") + mi::kHalfLog2Pi);\n"
          << in << "pb" << S << " |= !(" << sig << " > 0.0f);\n";
      }
    }
  };
  // one row (particle k): the pairs' accumulations, then the row's lp<s> / sl<j> scalars
  auto emit_acc_row = [&](const std::string& valid) {
    const char* in2 = "      ";
    for (int st = 0; st < g.num_sites; ++st) {
      const std::string S = site_str(st);
      if (g.sites[st].family == MI_NORMAL) {
        if (!normal_scale_const(st)) {   // per-particle sigma: this row's factors
          const std::string sig = role_expr(st, 1);
          o << in2 << "const float iv" << S << " = mi::rcp(" << sig << "), iq" << S << " = iv" << S
            << " * iv" << S << ";\n" << in2 << "const float lc" << S << " = -(logf(" << sig
            << ") + mi::kHalfLog2Pi);\n" << in2 << "pb" << S << " |= !(" << sig << " > 0.0f);\n";
        }
        o << in2 << "mi::f2 qa" << S << " = mi::splat2(-0.0f);\n";
        if (normal_needs_q1(st)) o << in2 << "mi::f2 qb" << S << " = mi::splat2(-0.0f);\n";
        o << in2 << "const float kl" << S << " = scale" << S << " * iq" << S << ";\n";
      } else {
        o << in2 << "mi::f2 qa" << S << " = mi::splat2(-0.0f);\n";
        if (role_grad(st, 0) == MI_GRAD_PARTICLE) o << in2 << "mi::f2 qb" << S << " = mi::splat2(-0.0f);\n";
      }
    }
    for (int op = 0; op < g.num_operands; ++op)
      if (dense_grad(op)) o << in2 << "mi::f2 g" << op << "[" << E / 2 << "];\n";
    o << in2 << "#pragma unroll\n" << in2 << "for (int h = 0; h < " << E / 2 << "; ++h) {\n";
    const std::string in3 = std::string(in2) + "  ";
    for (int op = 0; op < g.num_operands; ++op)
      if (dense_grad(op)) o << in3 << "g" << op << "[h] = mi::splat2(-0.0f);\n";
    for (int st = 0; st < g.num_sites; ++st) {
      const std::string S = site_str(st);
      const mi_site& site = g.sites[st];
      const std::string obs = site_obs(st, valid);
      const bool all = obs == "true";
      const std::string o0 = at_pair(obs, 0), o1 = at_pair(obs, 1);
      auto sel = [&](const std::string& x) {
        return all ? x : "mi::f2{" + o0 + " ? " + x + ".x : 0.0f, " + o1 + " ? " + x + ".y : 0.0f}";
      };
      const std::string V = pair_role(role_expr(st, 2));
      o << in3 << "{\n";
      if (site.family == MI_NORMAL) {
        const std::string L = pair_role(role_expr(st, 0));
        o << in3 << "  const mi::f2 lv = " << L << ", vv = " << V << ";\n";
        o << in3 << "  const mi::f2 df = vv - lv;\n";
        o << in3 << "  const mi::f2 t = " << sel("df") << ";\n";
        o << in3 << "  qa" << S << " = mi::fma2(t, t, qa" << S << ");\n";
        if (normal_needs_q1(st)) o << in3 << "  qb" << S << " = qb" << S << " + t;\n";
        o << in3 << "  pb" << S << " |= (lv.x != lv.x) | (lv.y != lv.y);\n";
        o << in3 << "  sb" << S << " |= (" << o0 << " & (vv.x != vv.x)) | (" << o1 << " & (vv.y != vv.y));\n";
        if (role_grad(st, 0) == MI_GRAD_DENSE)
          o << in3 << "  g" << site.operand[0] << "[h] = mi::fma2(mi::splat2(kl" << S << "), t, g"
            << site.operand[0] << "[h]);\n";
        if (role_grad(st, 2) == MI_GRAD_DENSE)
          o << in3 << "  g" << site.operand[2] << "[h] = mi::fma2(mi::splat2(-kl" << S << "), t, g"
            << site.operand[2] << "[h]);\n";
      } else {   // MI_BERNOULLI_LOGITS
        const std::string L = pair_role(role_expr(st, 0));
        o << in3 << "  const mi::f2 l = " << L << ", vv = " << V << ";\n";
        o << in3 << "  const mi::f2 t = mi::f2{mi::fast_exp(-fabsf(l.x)), mi::fast_exp(-fabsf(l.y))};\n";
        o << in3 << "  const mi::f2 u = 1.0f + t;\n";
        o << in3 << "  const mi::f2 r = mi::f2{mi::rcp(u.x), mi::rcp(u.y)};\n";
        o << in3 << "  const mi::f2 lu = mi::f2{__builtin_amdgcn_logf(u.x), __builtin_amdgcn_logf(u.y)};\n";
        o << in3 << "  const mi::f2 a = mi::fma2(l, vv, -mi::f2{fmaxf(l.x, 0.0f), fmaxf(l.y, 0.0f)});\n";
        o << in3 << "  const mi::f2 lp = mi::fma2(lu, mi::splat2(-0.69314718055994531f), a);\n";
        o << in3 << "  qa" << S << " = qa" << S << " + " << sel("lp") << ";\n";
        if (role_grad(st, 0) != MI_GRAD_NONE) {
          o << in3 << "  const mi::f2 tr = t * r;\n";
          o << in3 << "  const mi::f2 dd = vv - mi::f2{l.x >= 0.0f ? r.x : tr.x, l.y >= 0.0f ? r.y : tr.y};\n";
          o << in3 << "  const mi::f2 ds = " << sel("dd") << ";\n";
          if (role_grad(st, 0) == MI_GRAD_DENSE)
            o << in3 << "  g" << site.operand[0] << "[h] = mi::fma2(mi::splat2(scale" << S << "), ds, g"
              << site.operand[0] << "[h]);\n";
          else
            o << in3 << "  qb" << S << " = qb" << S << " + ds;\n";
        }
        o << in3 << "  pb" << S << " |= (l.x != l.x) | (l.y != l.y);\n";
        o << in3 << "  sb" << S << " |= (" << o0 << " & !((vv.x == 0.0f) | (vv.x == 1.0f))) | (" << o1
          << " & !((vv.y == 0.0f) | (vv.y == 1.0f)));\n";
      }
      o << in3 << "}\n";
    }
    o << in2 << "}\n";
    // the row's values: lp<s> per site, sl<j> per slot
    for (int st = 0; st < g.num_sites; ++st) {
      const std::string S = site_str(st);
      if (g.sites[st].family == MI_NORMAL)
        o << in2 << "const float lp" << S << " = fmaf(-0.5f * iq" << S << ", qa" << S << ".x + qa" << S
          << ".y, cn" << S << " * lc" << S << ");\n";
      else
        o << in2 << "const float lp" << S << " = qa" << S << ".x + qa" << S << ".y;\n";
    }
    if (g.compute_grads)
      for (int j = 0; j < g.num_slots; ++j) {
        o << in2 << "float sl" << j << " = -0.0f;\n";
        for (int st = 0; st < g.num_sites; ++st) {
          const std::string S = site_str(st);
          const mi_site& site = g.sites[st];
          for (int q = 0; q < 3; ++q) {
            if (role_grad(st, q) != MI_GRAD_PARTICLE || g.operands[site.operand[q]].slot != j) continue;
            if (site.family == MI_NORMAL) {
              if (q == 0) o << in2 << "sl" << j << " = fmaf(kl" << S << ", qb" << S << ".x + qb" << S << ".y, sl" << j << ");\n";
              else if (q == 2) o << in2 << "sl" << j << " = fmaf(-kl" << S << ", qb" << S << ".x + qb" << S << ".y, sl" << j << ");\n";
              else o << in2 << "sl" << j << " = fmaf(scale" << S << ", (iq" << S << " * (qa" << S << ".x + qa" << S
                     << ".y) - cn" << S << ") * iv" << S << ", sl" << j << ");\n";
            } else if (q == 0) {
              o << in2 << "sl" << j << " = fmaf(scale" << S << ", qb" << S << ".x + qb" << S << ".y, sl" << j << ");\n";
            }
          }
        }
      }
  };

  // Row loop with a fused guide draw (mi_draw): lane `lane` owns the element quads
  // base/4 + qq * 64 + lane (qq < E / 4), i.e. elements base + qq * 256 + lane * 4 + j, so that one
  // Philox call yields the lane's four normals of a quad -- exactly the eps of mi_normal_rsample for
  // (quad, particle). z = loc + eps * scale is formed in registers and d/dz is reduced over the
  // block's particles into dloc / dscale, so neither z nor dz touches memory.
  auto emit_draw_loop = [&]() {
    const char* in = "    ";
    auto elem = [&](const char* e) {
      return std::string("((") + e + " >> 2) * 256 + lane * 4 + (" + e + " & 3))";
    };
    o << in << "const long nominal = " << (plan.block_rows ? "seg_c" : "seg") << " * " << 64 * E
      << "L;\n";
    o << in << "const long shift = max(0L, nominal + " << 64 * E << "L - N);\n";
    o << in << "const long base = nominal - shift;\n";
    o << in << "bool ok[" << E << "];\n#pragma unroll\n" << in << "for (int e = 0; e < " << E
      << "; ++e) ok[e] = " << (plan.block_rows ? "live && " : "") << elem("e") << " >= shift;\n";
    for (int op = 0; op < g.num_operands; ++op)
      if (is(op, kShared))
        o << in << "float s" << op << "[" << E << "];\n" << in << "{ const float* __restrict__ r = x"
          << op << " + base + lane * 4;\n#pragma unroll\n" << in << "for (int e = 0; e < " << E
          << "; ++e) s" << op << "[e] = r[(e >> 2) * 256 + (e & 3)]; }\n";
    for (int st = 0; st < g.num_sites; ++st)
      if (mask_is(st, kShared))
        o << in << "bool m" << st << "[" << E << "];\n" << in
          << "{ const unsigned char* __restrict__ r = mk" << st
          << " + base + lane * 4;\n#pragma unroll\n" << in << "for (int e = 0; e < " << E
          << "; ++e) m" << st << "[e] = r[(e >> 2) * 256 + (e & 3)] != 0; }\n";
    o << in << "float dwl[" << E << "], dws[" << E << "];\n#pragma unroll\n" << in
      << "for (int e = 0; e < " << E << "; ++e) { const long i = base + " << elem("e")
      << "; dwl[e] = G.draw.loc[i * G.draw.loc_stride]; ";
    if (g.draw.scale_exp != nullptr)   // the guide's exp transform here; block row 0 writes it
      o << "dws[e] = expf(G.draw.scale_exp[i * G.draw.scale_stride]); if (blockIdx.y == 0 && ok[e]) "
           "const_cast<float*>(G.draw.scale)[i * G.draw.scale_stride] = dws[e]; }\n";
    else
      o << "dws[e] = G.draw.scale[i * G.draw.scale_stride]; }\n";
    const bool dgrad = g.compute_grads != 0;
    if (dgrad)
      o << in << "float dal[" << E << "], das[" << E << "];\n#pragma unroll\n" << in
        << "for (int e = 0; e < " << E << "; ++e) dal[e] = das[e] = 0.0f;\n";
    for (int op = 0; op < g.num_operands; ++op)
      if (is(op, kParticle) && op != pdraw)
        o << in << "float pn" << op << " = k_begin < k_end ? x" << op << "[k_begin * sk" << op
          << "] : 0.0f;\n";
    if (pdraw >= 0) {
      // the per-particle draw (mi_group.pdraw): this particle block's values into an LDS table,
      // each by one thread -- the normals and fmaf of mi_normal_rsample for (particle, element 0)
      // -- written to the operand by column block 0
      const std::string P = std::to_string(pdraw);
      o << in << "__shared__ float pdv[" << kPdrawTable << "];\n";
      o << in << "{\n";
      o << in << "  const unsigned long long pstep = G.pdraw.step + (G.pdraw.step_device != nullptr ? "
           "*G.pdraw.step_device : 0ull);\n";
      o << in << "  const float ploc = G.pdraw.loc[0];\n";
      o << in << "  const float psd = G.pdraw.scale_exp != nullptr ? expf(G.pdraw.scale_exp[0]) : "
           "G.pdraw.scale[0];\n";
      o << in << "  if (G.pdraw.scale_exp != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && "
           "threadIdx.x == 0) const_cast<float*>(G.pdraw.scale)[0] = psd;\n";
      o << in << "  for (long j = threadIdx.x; j < k_end - k_begin; j += 256) {\n";
      o << in << "    float pe[4];\n";
      o << in << "    mi::guide_normals(G.pdraw.seed, pstep, G.pdraw.stream_id, (unsigned long long)"
           "(G.pdraw.element_offset >> 2), (unsigned long long)(G.pdraw.particle_offset + k_begin + j), "
           "pe);\n";
      o << in << "    const float v = fmaf(pe[0], psd, ploc);\n";
      o << in << "    pdv[j] = v;\n";
      o << in << "    if (blockIdx.x == 0) const_cast<float*>(x" << P << ")[(k_begin + j) * sk" << P
        << "] = v;\n";
      o << in << "  }\n";
      o << in << "  __syncthreads();\n";
      o << in << "}\n";
    }
    // Two copies of the particle loop: a segment that is neither ragged nor past the end has
    // every element valid, and its unmasked sites need no per-element select.
    const bool acc = packed && acc_form(g, draw);
    // Two particles per iteration (accumulator form): the loop body below is emitted twice, for
    // particles k0 and k0 + 1, each in its own scope with `k` bound to its particle, so the two
    // Philox -> Box-Muller -> density chains are independent and the compiler interleaves them
    // (one chain per wave left half the issue cycles stalled at 4 waves per SIMD). An odd last
    // particle is evaluated twice and its second copy masked out of every sum (its tile row is
    // past the flush bound, its d loc / d scale terms are zeroed through an opaque lane mask: a
    // select on the uniform `two` became a branch around the gradient terms, which split the loop
    // body and kept the two chains from interleaving). Sums keep the sequential order:
    // dal / das add particle k0's terms, then k0 + 1's.
    const bool pairs = acc && draw_pairs() && tile_rows % 2 == 0;
    auto emit_k_loop = [&](const std::string& valid) {
    if (acc) emit_acc_prologue(valid);
    if (pairs) {
      for (int op = 0; op < g.num_operands; ++op)
        if (is(op, kParticle) && op != pdraw)
          o << in << "float pnn" << op << " = k_begin + 1 < k_end ? x" << op << "[(k_begin + 1) * sk"
            << op << "] : pn" << op << ";\n";
      o << in << "for (long k0 = k_begin; k0 < k_end; k0 += 2) {\n";
      o << in << "  const bool two = k0 + 1 < k_end;\n";
      o << in << "  const int r0 = (int)((k0 - k_begin) & " << tile_rows - 1 << ");\n";
      for (int op = 0; op < g.num_operands; ++op)
        if (is(op, kParticle) && op != pdraw) {
          // (pka / pkb: "pb<s>" names the sites' parameter flags)
          o << in << "  const float pka" << op << " = pn" << op << ", pkb" << op << " = pnn" << op
            << ";\n";
          o << in << "  if (k0 + 2 < k_end) { pn" << op << " = x" << op << "[(k0 + 2) * sk" << op
            << "]; pnn" << op << " = x" << op << "[min(k0 + 3, k_end - 1) * sk" << op << "]; }\n";
        }
      for (int v = 0; v < nv; ++v) o << in << "  float va" << v << ", vb" << v << ";\n";
    } else {
    o << in << "for (long k = k_begin; k < k_end; ++k) {\n";
    o << in << "  const int r = (int)((k - k_begin) & " << tile_rows - 1 << ");\n";
    }
    for (int copy = 0; copy < (pairs ? 2 : 1); ++copy) {
    if (pairs)
      o << in << "  {\n" << in << "  const long k = " << (copy == 0 ? "k0" : "two ? k0 + 1 : k0")
        << ";\n";
    if (packed) {   // pairs: eps and z = loc + eps * scale on packed instructions
      o << in << "  mi::f2 ep2[" << E / 2 << "];\n#pragma unroll\n" << in << "  for (int qq = 0; qq < "
        << E / 4 << "; ++qq) mi::guide_normals2(dseed, dstep, dstream, (unsigned long long)((base >> 2) "
           "+ dqoff + qq * 64 + lane), (unsigned long long)(dpoff + k), ep2[2 * qq], ep2[2 * qq + 1]);\n";
      o << in << "  float ep[" << E << "], d" << draw << "[" << E << "];\n#pragma unroll\n" << in
        << "  for (int h = 0; h < " << E / 2 << "; ++h) { const mi::f2 z = mi::fma2(ep2[h], "
           "mi::f2{dws[2 * h], dws[2 * h + 1]}, mi::f2{dwl[2 * h], dwl[2 * h + 1]}); d" << draw
        << "[2 * h] = z.x; d" << draw << "[2 * h + 1] = z.y; ep[2 * h] = ep2[h].x; ep[2 * h + 1] = "
           "ep2[h].y; }\n";
    } else {
      o << in << "  float ep[" << E << "];\n#pragma unroll\n" << in << "  for (int qq = 0; qq < "
        << E / 4 << "; ++qq) mi::guide_normals(dseed, dstep, dstream, (unsigned long long)((base >> 2) "
           "+ dqoff + qq * 64 + lane), (unsigned long long)(dpoff + k), &ep[4 * qq]);\n";
      o << in << "  float d" << draw << "[" << E << "];\n#pragma unroll\n" << in
        << "  for (int e = 0; e < " << E << "; ++e) d" << draw << "[e] = fmaf(ep[e], dws[e], dwl[e]);\n";
    }
    for (int op = 0; op < g.num_operands; ++op)
      if (op != draw && is(op, kDense))
        o << in << "  float d" << op << "[" << E << "];\n" << in
          << "  { const float* __restrict__ r = x" << op << " + k * sk" << op
          << " + base + lane * 4;\n#pragma unroll\n" << in << "  for (int e = 0; e < " << E
          << "; ++e) d" << op << "[e] = r[(e >> 2) * 256 + (e & 3)]; }\n";
    // per-particle operands: next row's values loaded one iteration ahead (a scalar load waited
    // on right away would stall the wave for its L2 round trip every row)
    for (int op = 0; op < g.num_operands; ++op)
      if (is(op, kParticle) && op == pdraw)
        o << in << "  const float p" << op << " = pdv[k - k_begin];\n";
      else if (is(op, kParticle) && pairs)
        o << in << "  const float p" << op << " = " << (copy == 0 ? "pka" : "pkb") << op << ";\n";
      else if (is(op, kParticle))
        o << in << "  const float p" << op << " = pn" << op << ";\n" << in << "  if (k + 1 < k_end) pn"
          << op << " = x" << op << "[(k + 1) * sk" << op << "];\n";
    for (int st = 0; st < g.num_sites; ++st)
      if (mask_is(st, kParticle))
        o << in << "  const bool mp" << st << " = mk" << st << "[k * msk" << st << "] != 0;\n";
    const char* in2 = "      ";
    if (acc) {
      emit_acc_row(valid);
    } else {
    zero_accumulators("      ");
    if (packed) {   // element pairs on the packed fp32 instructions
      for (int op = 0; op < g.num_operands; ++op)
        if (dense_grad(op)) o << in2 << "mi::f2 g" << op << "[" << E / 2 << "];\n";
      o << in2 << "#pragma unroll\n" << in2 << "for (int h = 0; h < " << E / 2 << "; ++h) {\n";
      const std::string inner = std::string(in2) + "  ";
      for (int op = 0; op < g.num_operands; ++op)
        if (dense_grad(op)) o << inner << "g" << op << "[h] = mi::splat2(0.0f);\n";
      for (int st = 0; st < g.num_sites; ++st) emit_site_eval2(o, g, st, valid, inner.c_str());
      o << in2 << "}\n";
    } else {
      for (int op = 0; op < g.num_operands; ++op)
        if (dense_grad(op)) o << in2 << "float g" << op << "[" << E << "];\n";
      o << in2 << "#pragma unroll\n" << in2 << "for (int e = 0; e < " << E << "; ++e) {\n";
      const std::string inner = std::string(in2) + "  ";
      for (int op = 0; op < g.num_operands; ++op)
        if (dense_grad(op)) o << inner << "g" << op << "[e] = 0.0f;\n";
      for (int st = 0; st < g.num_sites; ++st) emit_site_eval(o, g, st, valid, inner.c_str());
      o << in2 << "}\n";
    }
    }
    // g<op>[e] of either form
    auto gel = [&](int op, const char* e) {
      return packed ? "g" + std::to_string(op) + "[(" + e + ") >> 1][(" + e + ") & 1]"
                         : "g" + std::to_string(op) + "[" + e + "]";
    };
    if (pairs && copy == 1)   // (an odd last particle's second copy adds nothing)
      for (int op = 0; op < g.num_operands; ++op)
        if (dense_grad(op))
          o << in2 << "#pragma unroll\n" << in2 << "for (int h = 0; h < " << E / 2 << "; ++h) g" << op
            << "[h] = mi::f2{mi::keep_if(g" << op << "[h].x, two), mi::keep_if(g" << op
            << "[h].y, two)};\n";
    for (int op = 0; op < g.num_operands; ++op) {
      if (!dense_grad(op)) continue;
      if (op == draw && packed)
        o << in2 << "#pragma unroll\n" << in2 << "for (int h = 0; h < " << E / 2
          << "; ++h) { const mi::f2 a = mi::f2{dal[2 * h], dal[2 * h + 1]} + g" << op
          << "[h]; const mi::f2 b = mi::fma2(g" << op << "[h], mi::f2{ep[2 * h], ep[2 * h + 1]}, "
             "mi::f2{das[2 * h], das[2 * h + 1]}); dal[2 * h] = a.x; dal[2 * h + 1] = a.y; "
             "das[2 * h] = b.x; das[2 * h + 1] = b.y; }\n";
      else if (op == draw)
        o << in2 << "#pragma unroll\n" << in2 << "for (int e = 0; e < " << E << "; ++e) { dal[e] += g"
          << op << "[e]; das[e] = fmaf(g" << op << "[e], ep[e], das[e]); }\n";
      else
        o << in2 << "{ float* __restrict__ r = gx" << op << " + k * gsk" << op
          << " + base + lane * 4;\n#pragma unroll\n" << in2 << "for (int e = 0; e < " << E
          << "; ++e) if (ok[e]) r[(e >> 2) * 256 + (e & 3)] = G.grad_scale * " << gel(op, "e")
          << "; }\n";
    }
    if (!pairs) {
      emit_particle_sums(in2, plan.block_rows);
    } else {
      for (int v = 0; v < nv; ++v)
        o << in2 << (copy == 0 ? "va" : "vb") << v << " = " << value_expr(v) << ";\n";
      o << in << "  }\n";
    }
    }   // copies
    if (pairs) {
      // particle k0's row r0, k0 + 1's row r0 + 1; the flush sees the last particle written
      const char* in2 = "      ";
      for (int v = 0; v < nv; ++v)
        o << in2 << "tile[" << v * tile_rows * 65 << " + r0 * 65 + lane] = va" << v << ";\n" << in2
          << "tile[" << v * tile_rows * 65 << " + (r0 + 1) * 65 + lane] = vb" << v << ";\n";
      o << in2 << "{\n" << in2 << "const int r = two ? r0 + 1 : r0;\n" << in2
        << "const long k = two ? k0 + 1 : k0;\n";
      emit_particle_sums(in2, plan.block_rows, false);
      o << in2 << "}\n";
    }
    o << in << "}\n";
    };
    o << in << "if (" << (plan.block_rows ? "live && " : "") << "shift == 0) {\n";
    emit_k_loop("true");
    o << in << "} else {\n";
    emit_k_loop("ok[e]");
    o << in << "}\n";
    if (dgrad)
      o << in << "#pragma unroll\n" << in << "for (int e = 0; e < " << E << "; ++e) if (ok[e]) {\n"
        << in << "  const long i = (long)blockIdx.y * N + base + " << elem("e") << ";\n"
        << in << "  G.draw.dloc[i] = G.grad_scale * dal[e];\n"
        << in << "  G.draw.dscale[i] = G.grad_scale * das[e];\n"
        << in << "}\n";
  };

  if (row && draw >= 0) {
    o << "  const unsigned long long dseed = G.draw.seed;\n";
    o << "  const unsigned long long dstep = G.draw.step + (G.draw.step_device != nullptr ? "
         "*G.draw.step_device : 0ull);\n";
    o << "  const unsigned dstream = G.draw.stream_id;\n";
    o << "  const long dpoff = G.draw.particle_offset;\n";
    o << "  const long dqoff = G.draw.element_offset >> 2;   // data-sharded draws\n";
    if (plan.block_rows) {
      // every wave runs the loop (block barriers at the flushes): a wave past the last segment
      // re-reads the last one with all of its elements masked off
      o << "  __shared__ float bsum[" << nv * 4 * tile_rows << "];\n";
      o << "  const bool live = seg < nseg;\n";
      o << "  {\n";
      o << "    const long seg_c = live ? seg : nseg - 1;\n";
    } else {
      o << "  if (seg < nseg) {\n";
    }
    o << "    const long k_begin = (long)blockIdx.y * arg;\n";
    o << "    const long k_end = min(K, k_begin + arg);\n";
    emit_draw_loop();
    o << "  }\n";
  } else if (row) {
    // Lane `lane` owns elements base + e * 64 + lane of each row (coalesced per e). When N spans
    // at least one whole segment, every segment is loaded as a whole one: the ragged last segment
    // is shifted back to end at N and masks the elements its predecessor already owns (`ok`), so
    // no load needs a bound and unit-stride operands use one row pointer with compile-time
    // offsets e * 64 folded into the instructions. Smaller N takes the clamped-index copy.
    o << "  if (seg < nseg) {\n";
    o << "    const long k_begin = (long)blockIdx.y * arg;\n";
    o << "    const long k_end = min(K, k_begin + arg);\n";
    if (g.N >= 64L * E) {
      o << "    const long nominal = seg * " << 64 * E << "L;\n";
      o << "    const long shift = max(0L, nominal + " << 64 * E << "L - N);\n";
      o << "    const long base = nominal - shift;\n";
      emit_row_loop(true);
    } else {
      o << "    const long base = seg * " << 64 * E << "L;\n";
      emit_row_loop(false);
    }
    o << "  }\n";
  } else {
    const int kw = plan.kw;
    const int istep = 64 / kw;
    o << "  const int kq = lane & " << (kw - 1) << ";\n";
    o << "  const int isub = lane / " << kw << ";\n";
    o << "  const long k = (long)blockIdx.y * " << kw << " + kq;\n";
    o << "  const bool kok = k < K;\n";
    o << "  const long kc = kok ? k : K - 1;\n";
    zero_accumulators("  ");
    o << "  if (seg < nseg) {\n";
    particle_loads("    ", "kc");
    o << "    const long i_begin = seg * arg;\n";
    o << "    const long i_end = min(N, i_begin + arg);\n";
    o << "    for (long i0 = i_begin + isub; i0 < i_end; i0 += " << E * istep << ") {\n";
    o << "      long ii[" << E << "]; bool okv[" << E << "];\n";
    o << "#pragma unroll\n      for (int e = 0; e < " << E << "; ++e) { const long i = i0 + e * "
      << istep << "; okv[e] = kok && i < i_end; ii[e] = i < i_end ? i : i_end - 1; }\n";
    for (int op = 0; op < g.num_operands; ++op)
      if (is(op, kShared))
        o << "      float s" << op << "[" << E << "];\n#pragma unroll\n      for (int e = 0; e < " << E
          << "; ++e) s" << op << "[e] = x" << op << "[ii[e] * si" << op << "];\n";
    for (int s = 0; s < g.num_sites; ++s)
      if (mask_is(s, kShared))
        o << "      bool m" << s << "[" << E << "];\n#pragma unroll\n      for (int e = 0; e < " << E
          << "; ++e) m" << s << "[e] = mk" << s << "[ii[e] * msi" << s << "] != 0;\n";
    declare_dense("      ", "d");
    dense_loads("      ", "d", "kc", "ii[e]");
    compute_and_store("      ", "okv[e]", "kc", "ii[e]");
    o << "    }\n  }\n";
    std::vector<std::string> finals;
    for (int v = 0; v < nv; ++v) {
      o << "  float fin" << v << " = " << value_expr(v) << ";\n";
      if (kw < 64) o << "  fin" << v << " = mi::wave_sum_strided(fin" << v << ", " << kw << ");\n";
    }
    o << "  if (seg < nseg && kok && isub == 0) {\n";
    for (int v = 0; v < nv; ++v)
      o << "    part[((long)" << v << " * nseg + seg) * K + k] = fin" << v << ";\n";
    o << "  }\n";
  }
  // dense masks use the names "dm<s>" inside rows; map mask_var's "md<s>[e]" onto them
  for (int s = 0; s < g.num_sites; ++s)
    o << "  mi::publish_flags(flags + " << s << ", (pb" << s << " ? " << MI_FLAG_PARAM << "u : 0u) | (sb"
      << s << " ? " << MI_FLAG_SUPPORT << "u : 0u));\n";
  o << "  mi::span_end(G.stamps, span_t0);\n";
  o << "}\n";
  std::string text = o.str();
  for (int s = 0; s < g.num_sites; ++s) {
    const std::string from = "md" + std::to_string(s) + "[e]", to = "dm" + std::to_string(s) + "[e]";
    for (size_t at = text.find(from); at != std::string::npos; at = text.find(from, at + to.size()))
      text.replace(at, from.size(), to);
  }
  return text;
}

// ---- compile cache ---------------------------------------------------------------------------

struct Compiled {
  hipModule_t module = nullptr;
  hipFunction_t function = nullptr;
  bool failed = false;
};

std::mutex g_mutex;
std::map<std::string, Compiled> g_cache;

bool jit_disabled() {
  const char* v = std::getenv("MININF_AMD_JIT");
  return v != nullptr && (std::strcmp(v, "0") == 0 || std::strcmp(v, "off") == 0);
}

bool compile_only(const std::string& source, std::vector<char>* code, std::string* log) {
  hiprtcProgram prog;
  const char* headers[] = {kHeaderText, kMathText, kStddefStub};
  const char* names[] = {"mininf_amd.h", "device_math.hpp", "stddef.h"};
  if (hiprtcCreateProgram(&prog, source.c_str(), "mi_site_program.hip", 3, headers, names) !=
      HIPRTC_SUCCESS)
    return false;
  const char* options[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize"};
  const hiprtcResult rc = hiprtcCompileProgram(prog, 4, options);
  if (log != nullptr) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    log->assign(n, '\0');
    if (n > 0) hiprtcGetProgramLog(prog, log->data());
  }
  if (rc == HIPRTC_SUCCESS && code != nullptr) {
    size_t size = 0;
    hiprtcGetCodeSize(prog, &size);
    code->resize(size);
    hiprtcGetCode(prog, code->data());
  }
  hiprtcDestroyProgram(&prog);
  return rc == HIPRTC_SUCCESS;
}

Compiled compile(const std::string& source) {
  Compiled out;
  std::vector<char> code;
  std::string log;
  if (const char* dir = std::getenv("MININF_AMD_JIT_DUMP")) {   // diagnostics: keep the source
    static int serial = 0;
    const std::string path = std::string(dir) + "/site_program_" + std::to_string(serial++) + ".hip";
    if (FILE* f = fopen(path.c_str(), "w")) {
      fwrite(source.data(), 1, source.size(), f);
      fclose(f);
    }
  }
  if (!compile_only(source, &code, &log)) {
    if (std::getenv("MININF_AMD_JIT_VERBOSE") != nullptr)
      fprintf(stderr, "mininf_amd: site program failed to compile:\n%s\n%s\n", log.c_str(),
              source.c_str());
    out.failed = true;
    return out;
  }
  if (hipModuleLoadData(&out.module, code.data()) != hipSuccess ||
      hipModuleGetFunction(&out.function, out.module, "mi_site_program") != hipSuccess) {
    out.failed = true;
  }
  return out;
}

}  // namespace

std::string mi_jit_source(const mi_group& g, const PlanInfo& plan) { return generate(g, plan); }

int mi_jit_launch(const mi_group& g, const PlanInfo& plan, float* part, int64_t nseg, int64_t arg,
                  uint32_t* flags, hipStream_t stream) {
  if (jit_disabled()) return 1;
  const std::string key = signature(g, plan).text;
  hipFunction_t fn = nullptr;
  {
    std::lock_guard<std::mutex> lock(g_mutex);
    auto it = g_cache.find(key);
    if (it == g_cache.end()) it = g_cache.emplace(key, compile(generate(g, plan))).first;
    if (it->second.failed) return 1;
    fn = it->second.function;
  }
  mi_group G = g;
  long nseg_l = (long)nseg, arg_l = (long)arg;
  void* args[] = {&G, &part, &nseg_l, &arg_l, &flags};
  const hipError_t e = hipModuleLaunchKernel(fn, plan.grid_x, plan.grid_y, 1, 256, 1, 1, 0, stream,
                                             args, nullptr);
  return e == hipSuccess ? 0 : -(int)e;
}

bool mi_jit_compile_check(const mi_group& g, const PlanInfo& plan, std::string* log) {
  return compile_only(generate(g, plan), nullptr, log);
}

bool mi_jit_enabled() { return !jit_disabled(); }

size_t mi_jit_cache_size() {
  std::lock_guard<std::mutex> lock(g_mutex);
  return g_cache.size();
}
