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
    default: return "eval_beta";
  }
}

bool role_used(int family, int q) {
  return !((family == MI_BERNOULLI_LOGITS || family == MI_BERNOULLI_PROBS) && q == 1);
}

// Everything about a group that changes the generated code.
struct Signature {
  std::string text;
};

std::string operand_var(const mi_group& g, int o, bool row_layout) {
  const Kind k = kind_of(g.operands[o].stride_k, g.operands[o].stride_i);
  std::ostringstream s;
  switch (k) {
    case kBroadcast: s << "b" << o; break;
    case kShared: s << (row_layout ? "s" : "sv") << o << (row_layout ? "[e]" : ""); break;
    case kParticle: s << "p" << o; break;
    default: s << "d" << o; break;
  }
  return s.str();
}

std::string mask_kind_tag(const mi_site& st) {
  if (st.mask == nullptr) return "-";
  return std::to_string((int)kind_of(st.mask_stride_k, st.mask_stride_i));
}

Signature signature(const mi_group& g, const PlanInfo& plan) {
  std::ostringstream s;
  s << (plan.row ? "R" : "C") << plan.elems << "/" << plan.kw << "|" << g.num_operands << ":";
  for (int o = 0; o < g.num_operands; ++o) {
    const mi_operand& op = g.operands[o];
    s << (int)kind_of(op.stride_k, op.stride_i) << (g.compute_grads ? op.grad_mode : 0)
      << (op.grad_mode == MI_GRAD_PARTICLE ? op.slot : 0) << ",";
  }
  s << "|" << g.num_sites << ":";
  for (int i = 0; i < g.num_sites; ++i) {
    const mi_site& st = g.sites[i];
    s << st.family << "(" << st.operand[0] << "," << st.operand[1] << "," << st.operand[2] << ","
      << mask_kind_tag(st) << ")";
  }
  s << "|" << g.num_slots << "|" << g.compute_grads;
  return Signature{s.str()};
}

// ---- source generation ----------------------------------------------------------------------

void emit_site_eval(std::ostringstream& o, const mi_group& g, int s, bool row_layout,
                    const char* valid) {
  const mi_site& st = g.sites[s];
  std::string r[3];
  for (int q = 0; q < 3; ++q) {
    if (!role_used(st.family, q)) {
      r[q] = "0.0f";
    } else if (st.operand[q] < 0) {
      r[q] = "c" + std::to_string(s) + "_" + std::to_string(q);
    } else {
      r[q] = operand_var(g, st.operand[q], row_layout);
    }
  }
  o << "        {\n          mi::Elem el;\n";
  if (st.family == MI_BERNOULLI_LOGITS || st.family == MI_BERNOULLI_PROBS)
    o << "          mi::" << eval_fn(st.family) << "(" << r[0] << ", " << r[2] << ", el);\n";
  else
    o << "          mi::" << eval_fn(st.family) << "(" << r[0] << ", " << r[1] << ", " << r[2]
      << ", el);\n";
  std::string obs = valid;
  if (st.mask != nullptr) {
    const Kind mk = kind_of(st.mask_stride_k, st.mask_stride_i);
    std::string m;
    if (mk == kBroadcast) m = "m" + std::to_string(s);
    else if (mk == kShared) m = row_layout ? "m" + std::to_string(s) + "[e]" : "mv" + std::to_string(s);
    else if (mk == kParticle) m = "mp" + std::to_string(s);
    else m = "md" + std::to_string(s);
    obs = "(" + obs + " && " + m + ")";
  }
  o << "          const bool obs = " << obs << ";\n";
  o << "          lp" << s << " += obs ? el.lp : 0.0f;\n";
  o << "          fl" << s << " |= (el.param_bad ? " << MI_FLAG_PARAM
    << "u : 0u) | ((obs && el.support_bad) ? " << MI_FLAG_SUPPORT << "u : 0u);\n";
  if (g.compute_grads) {
    bool any = false;
    for (int q = 0; q < 3; ++q) {
      const int op = st.operand[q];
      if (op >= 0 && role_used(st.family, q) && g.operands[op].grad_mode != MI_GRAD_NONE) any = true;
    }
    if (any) o << "          const float w = obs ? scale" << s << " : 0.0f;\n";
    for (int q = 0; q < 3; ++q) {
      const int op = st.operand[q];
      if (op < 0 || !role_used(st.family, q)) continue;
      if (g.operands[op].grad_mode == MI_GRAD_DENSE)
        o << "          g" << op << " = fmaf(w, el.d[" << q << "], g" << op << ");\n";
      else if (g.operands[op].grad_mode == MI_GRAD_PARTICLE)
        o << "          sl" << g.operands[op].slot << " = fmaf(w, el.d[" << q << "], sl"
          << g.operands[op].slot << ");\n";
    }
  }
  o << "        }\n";
}

std::string generate(const mi_group& g, const PlanInfo& plan) {
  const bool row = plan.row;
  const int E = plan.elems;
  std::ostringstream o;
  o << "#include \"device_math.hpp\"\n";
  o << "extern \"C\" __global__ __launch_bounds__(256) void mi_site_program(const mi_group G, "
       "float* __restrict__ part, long nseg, long arg, unsigned* __restrict__ flags) {\n";
  o << "  const int lane = threadIdx.x & 63;\n";
  o << "  const long seg = (long)blockIdx.x * 4 + (threadIdx.x >> 6);\n";
  o << "  const long K = G.K, N = G.N;\n";
  for (int s = 0; s < g.num_sites; ++s) {
    o << "  unsigned fl" << s << " = 0u;\n";
    o << "  const float scale" << s << " = (float)G.sites[" << s << "].scale;\n";
    for (int q = 0; q < 3; ++q)
      if (g.sites[s].operand[q] < 0 && role_used(g.sites[s].family, q))
        o << "  const float c" << s << "_" << q << " = G.sites[" << s << "].constant[" << q << "];\n";
  }
  // Pointers and strides as locals (scalar registers).
  for (int op = 0; op < g.num_operands; ++op) {
    o << "  const float* __restrict__ x" << op << " = G.operands[" << op << "].data;\n";
    o << "  const long sk" << op << " = G.operands[" << op << "].stride_k, si" << op
      << " = G.operands[" << op << "].stride_i;\n";
    if (g.compute_grads && g.operands[op].grad_mode == MI_GRAD_DENSE) {
      o << "  float* __restrict__ gx" << op << " = G.operands[" << op << "].grad;\n";
      o << "  const long gsk" << op << " = G.operands[" << op << "].grad_stride_k, gsi" << op
        << " = G.operands[" << op << "].grad_stride_i;\n";
    }
    if (kind_of(g.operands[op].stride_k, g.operands[op].stride_i) == kBroadcast)
      o << "  const float b" << op << " = x" << op << "[0];\n";
  }
  for (int s = 0; s < g.num_sites; ++s) {
    if (g.sites[s].mask == nullptr) continue;
    o << "  const unsigned char* __restrict__ mk" << s << " = G.sites[" << s << "].mask;\n";
    o << "  const long msk" << s << " = G.sites[" << s << "].mask_stride_k, msi" << s
      << " = G.sites[" << s << "].mask_stride_i;\n";
    if (kind_of(g.sites[s].mask_stride_k, g.sites[s].mask_stride_i) == kBroadcast)
      o << "  const bool m" << s << " = mk" << s << "[0] != 0;\n";
  }
  const int nv = g.num_sites + (g.compute_grads ? g.num_slots : 0);
  auto zero_accumulators = [&](const char* indent) {
    for (int s = 0; s < g.num_sites; ++s) o << indent << "float lp" << s << " = 0.0f;\n";
    if (g.compute_grads)
      for (int j = 0; j < g.num_slots; ++j) o << indent << "float sl" << j << " = 0.0f;\n";
  };
  auto value_name = [&](int v) {
    return v < g.num_sites ? "lp" + std::to_string(v) : "sl" + std::to_string(v - g.num_sites);
  };
  auto dense_loads = [&](const char* indent, const char* kexpr, const char* iexpr) {
    for (int op = 0; op < g.num_operands; ++op)
      if (kind_of(g.operands[op].stride_k, g.operands[op].stride_i) == kDense)
        o << indent << "const float d" << op << " = x" << op << "[" << kexpr << " * sk" << op
          << " + " << iexpr << " * si" << op << "];\n";
    for (int s = 0; s < g.num_sites; ++s) {
      if (g.sites[s].mask == nullptr) continue;
      if (kind_of(g.sites[s].mask_stride_k, g.sites[s].mask_stride_i) == kDense)
        o << indent << "const bool md" << s << " = mk" << s << "[" << kexpr << " * msk" << s
          << " + " << iexpr << " * msi" << s << "] != 0;\n";
    }
    if (g.compute_grads)
      for (int op = 0; op < g.num_operands; ++op)
        if (g.operands[op].grad_mode == MI_GRAD_DENSE) o << indent << "float g" << op << " = 0.0f;\n";
  };
  auto dense_stores = [&](const char* indent, const char* guard, const char* kexpr,
                          const char* iexpr) {
    if (!g.compute_grads) return;
    for (int op = 0; op < g.num_operands; ++op)
      if (g.operands[op].grad_mode == MI_GRAD_DENSE)
        o << indent << "if (" << guard << ") gx" << op << "[" << kexpr << " * gsk" << op << " + "
          << iexpr << " * gsi" << op << "] = G.grad_scale * g" << op << ";\n";
  };
  auto particle_loads = [&](const char* indent, const char* kexpr) {
    for (int op = 0; op < g.num_operands; ++op)
      if (kind_of(g.operands[op].stride_k, g.operands[op].stride_i) == kParticle)
        o << indent << "const float p" << op << " = x" << op << "[" << kexpr << " * sk" << op << "];\n";
    for (int s = 0; s < g.num_sites; ++s)
      if (g.sites[s].mask != nullptr &&
          kind_of(g.sites[s].mask_stride_k, g.sites[s].mask_stride_i) == kParticle)
        o << indent << "const bool mp" << s << " = mk" << s << "[" << kexpr << " * msk" << s
          << "] != 0;\n";
  };

  if (row) {
    o << "  if (seg < nseg) {\n";
    o << "    const long base = seg * " << 64 * E << "L;\n";
    o << "    const long k_begin = (long)blockIdx.y * arg;\n";
    o << "    const long k_end = min(K, k_begin + arg);\n";
    o << "    long idx[" << E << "]; bool ok[" << E << "];\n";
    o << "#pragma unroll\n    for (int e = 0; e < " << E << "; ++e) { const long i = base + e * 64 + lane; "
         "ok[e] = i < N; idx[e] = ok[e] ? i : N - 1; }\n";
    // shared (per-element, particle-independent) operands and masks: loaded once per thread
    for (int op = 0; op < g.num_operands; ++op)
      if (kind_of(g.operands[op].stride_k, g.operands[op].stride_i) == kShared)
        o << "    float s" << op << "[" << E << "];\n#pragma unroll\n    for (int e = 0; e < " << E
          << "; ++e) s" << op << "[e] = x" << op << "[idx[e] * si" << op << "];\n";
    for (int s = 0; s < g.num_sites; ++s)
      if (g.sites[s].mask != nullptr &&
          kind_of(g.sites[s].mask_stride_k, g.sites[s].mask_stride_i) == kShared)
        o << "    bool m" << s << "[" << E << "];\n#pragma unroll\n    for (int e = 0; e < " << E
          << "; ++e) m" << s << "[e] = mk" << s << "[idx[e] * msi" << s << "] != 0;\n";
    o << "    for (long kb = k_begin; kb < k_end; kb += 64) {\n";
    for (int v = 0; v < nv; ++v) o << "      float keep" << v << " = 0.0f;\n";
    o << "      const int rows = (int)min(64L, k_end - kb);\n";
    o << "      for (int r = 0; r < rows; ++r) {\n";
    o << "        const long k = kb + r;\n";
    particle_loads("        ", "k");
    zero_accumulators("        ");
    o << "#pragma unroll\n        for (int e = 0; e < " << E << "; ++e) {\n";
    o << "          const long i = idx[e];\n";
    dense_loads("          ", "k", "i");
    for (int s = 0; s < g.num_sites; ++s) emit_site_eval(o, g, s, true, "ok[e]");
    dense_stores("          ", "ok[e]", "k", "i");
    o << "        }\n";
    for (int v = 0; v < nv; ++v)
      o << "        { const float t = mi::wave_sum(" << value_name(v) << "); keep" << v
        << " = (lane == r) ? t : keep" << v << "; }\n";
    o << "      }\n";
    o << "      if (lane < rows) {\n";
    for (int v = 0; v < nv; ++v)
      o << "        part[((long)" << v << " * nseg + seg) * K + kb + lane] = keep" << v << ";\n";
    o << "      }\n    }\n  }\n";
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
    o << "#pragma unroll " << E << "\n";
    o << "    for (long i = i_begin + isub; i < i_end; i += " << istep << ") {\n";
    for (int op = 0; op < g.num_operands; ++op)
      if (kind_of(g.operands[op].stride_k, g.operands[op].stride_i) == kShared)
        o << "      const float sv" << op << " = x" << op << "[i * si" << op << "];\n";
    for (int s = 0; s < g.num_sites; ++s)
      if (g.sites[s].mask != nullptr &&
          kind_of(g.sites[s].mask_stride_k, g.sites[s].mask_stride_i) == kShared)
        o << "      const bool mv" << s << " = mk" << s << "[i * msi" << s << "] != 0;\n";
    dense_loads("      ", "kc", "i");
    for (int s = 0; s < g.num_sites; ++s) emit_site_eval(o, g, s, false, "kok");
    dense_stores("      ", "kok", "kc", "i");
    o << "    }\n  }\n";
    if (kw < 64)
      for (int v = 0; v < nv; ++v)
        o << "  " << value_name(v) << " = mi::wave_sum_strided(" << value_name(v) << ", " << kw
          << ");\n";
    o << "  if (seg < nseg && kok && isub == 0) {\n";
    for (int v = 0; v < nv; ++v)
      o << "    part[((long)" << v << " * nseg + seg) * K + k] = " << value_name(v) << ";\n";
    o << "  }\n";
  }
  for (int s = 0; s < g.num_sites; ++s) o << "  mi::publish_flags(flags + " << s << ", fl" << s << ");\n";
  o << "}\n";
  return o.str();
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
  const char* options[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
  const hiprtcResult rc = hiprtcCompileProgram(prog, 3, options);
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

size_t mi_jit_cache_size() {
  std::lock_guard<std::mutex> lock(g_mutex);
  return g_cache.size();
}
