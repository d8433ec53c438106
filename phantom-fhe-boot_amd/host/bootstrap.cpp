#include "bootstrap.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <deque>
#include <exception>
#include <set>
#include <stdexcept>
#include <thread>

#include "../csrc/ckks.h"
#include "../csrc/rns.h"
#include "evaluate.h"
#include "numth.h"
#include "traffic.h"

namespace phantom {

// ======================================================================================
// host-side math
// ======================================================================================
namespace boot {

static std::complex<double> root_of_unity(uint64_t e, uint64_t M) {
  const double a = 2.0 * M_PI * static_cast<double>(e % M) / static_cast<double>(M);
  return {std::cos(a), std::sin(a)};
}

DiagMap stage(size_t n, int s, bool inverse) {
  const size_t m = size_t(1) << s, h = m / 2, M = 4 * n;
  if (m > n) throw std::invalid_argument("stage out of range");
  std::vector<uint64_t> pw(h);  // 5^j mod 4m
  uint64_t p5 = 1;
  for (size_t j = 0; j < h; ++j) {
    pw[j] = p5;
    p5 = p5 * 5 % (4 * m);
  }
  cvec d0(n), dp(n), dm(n);
  for (size_t p = 0; p < n; ++p) {
    const size_t j = p % m;
    if (j < h) {
      const std::complex<double> t = root_of_unity((n / m) * pw[j], M);
      d0[p] = inverse ? 0.5 : 1.0;
      dp[p] = inverse ? std::complex<double>(0.5) : t;
    } else {
      const std::complex<double> t = root_of_unity((n / m) * pw[j - h], M);
      if (inverse) {
        dm[p] = std::conj(t) * 0.5;
        d0[p] = -std::conj(t) * 0.5;
      } else {
        d0[p] = -t;
        dm[p] = 1.0;
      }
    }
  }
  DiagMap d;
  auto add = [&](int a, const cvec& v) {
    auto it = d.find(a);
    if (it == d.end()) {
      d.emplace(a, v);
    } else {
      for (size_t i = 0; i < n; ++i) it->second[i] += v[i];
    }
  };
  add(0, d0);
  add(static_cast<int>(h % n), dp);
  add(static_cast<int>((n - h) % n), dm);
  return d;
}

DiagMap compose(const DiagMap& A, const DiagMap& B, size_t n) {
  DiagMap out;
  for (const auto& [a, alpha] : A)
    for (const auto& [b, beta] : B) {
      const int key = static_cast<int>((static_cast<size_t>(a) + static_cast<size_t>(b)) % n);
      cvec& dst = out[key];
      if (dst.empty()) dst.assign(n, {0.0, 0.0});
      for (size_t p = 0; p < n; ++p) dst[p] += alpha[p] * beta[(p + a) % n];
    }
  return out;
}

DiagMap lift_blocks(const DiagMap& T, size_t n, size_t S, const cvec* out_mask, const cvec* in_mask) {
  if (S % n) throw std::invalid_argument("slot count not a multiple of the block size");
  DiagMap out;
  for (const auto& [a, d] : T) {
    for (size_t p = 0; p < S; ++p) {
      const size_t r = p % n;
      std::complex<double> v = d[r];
      if (v == std::complex<double>(0.0, 0.0)) continue;
      // the pair (p, p + a) of the n-dim map stays inside p's block: offset a or a - n
      const long off = r + static_cast<size_t>(a) < n ? static_cast<long>(a) : static_cast<long>(a) - static_cast<long>(n);
      const size_t key = static_cast<size_t>(((off % static_cast<long>(S)) + static_cast<long>(S)) % static_cast<long>(S));
      const size_t q = (p + key) % S;
      if (out_mask) v *= (*out_mask)[p % out_mask->size()];
      if (in_mask) v *= (*in_mask)[q % in_mask->size()];
      cvec& dst = out[static_cast<int>(key)];
      if (dst.empty()) dst.assign(S, {0.0, 0.0});
      dst[p] += v;
    }
  }
  return out;
}

cvec apply(const DiagMap& T, const cvec& v) {
  const size_t n = v.size();
  cvec out(n, {0.0, 0.0});
  for (const auto& [a, d] : T)
    for (size_t p = 0; p < n; ++p) out[p] += d[p] * v[(p + a) % n];
  return out;
}

std::vector<double> chebyshev_coefficients(double (*f)(double, const double*), const double* args, int degree) {
  const int n = degree + 1;
  std::vector<double> fx(n), c(n, 0.0);
  for (int j = 0; j < n; ++j) fx[j] = f(std::cos(M_PI * (j + 0.5) / n), args);
  for (int k = 0; k < n; ++k) {
    double acc = 0.0;
    for (int j = 0; j < n; ++j) acc += fx[j] * std::cos(M_PI * k * (j + 0.5) / n);
    c[k] = 2.0 * acc / n;
  }
  c[0] *= 0.5;
  return c;
}

double scaled_cosine(double y, const double* args) {
  const double K = args[0], r = args[1], two_r = std::pow(2.0, r);
  return std::pow(2.0 * M_PI, -1.0 / two_r) * std::cos(2.0 * M_PI * (K * y - 0.25) / two_r);
}

}  // namespace boot

// ======================================================================================
// Chebyshev evaluation: p = q T_m + r recursion down to degree < 16 leaves
// ======================================================================================
namespace {

constexpr int kLeafDegree = 15;
static_assert(kLeafDegree <= phx::kLeafMaxK, "leaf degree above the leaf kernel's input count");

int ceil_log2(int x) {
  int r = 0;
  while ((1 << r) < x) ++r;
  return r;
}

// the split p = q T_m + r of a degree-d series (d > kLeafDegree): the largest power of two m
// with 2m <= d, halved when d is itself a power of two so that q is never a constant
int cheb_split(int d) {
  int m = 1;
  while (2 * m <= d) m *= 2;
  return m == d ? m / 2 : m;
}

// depth (levels consumed) of evaluating a degree-d series with the recursion below
int cheb_depth(int d) {
  if (d <= kLeafDegree) return (d <= 1 ? 0 : ceil_log2(d)) + 1;
  const int m = cheb_split(d);
  return std::max(std::max(cheb_depth(d - m), ceil_log2(m)) + 1, cheb_depth(m - 1));
}

// The evaluator runs B independent series inputs ("lanes", all at one level and scale) in lockstep:
// EvalMod evaluates the same series on the real and the imaginary half of the CoeffToSlot output,
// so every product of the two halves shares one key switch launch sequence (MulAddRescaleBatch),
// and the members of a power-ladder generation do too.
using Lanes = std::vector<PhantomCiphertext>;

struct ChebEvaluator {
  const PhantomContext& cc;
  const PhantomRelinKey& rlk;
  const std::vector<double>& sf;
  LeafTableCache& tables;
  size_t B = 1;
  std::map<int, Lanes> T;
  std::map<std::pair<int, size_t>, Lanes> aligned_;  // T_i brought to a deeper level

  static size_t lvl(const Lanes& v) { return level_of(v.at(0)); }

  // T_i at level `l` (>= its own), cached: the power ladder re-uses T_1, T_2, .. at the level of
  // every larger factor
  const Lanes& aligned(int i, size_t l) {
    const Lanes& t = get(i);
    if (lvl(t) == l) return t;
    auto key = std::make_pair(i, l);
    auto it = aligned_.find(key);
    if (it != aligned_.end()) return it->second;
    Lanes v(B);
    for (size_t b = 0; b < B; ++b) {
      PhantomCiphertext tmp;
      const PhantomCiphertext& r = AtLevel(cc, t[b], l, sf, tmp);
      v[b] = &r == &t[b] ? PhantomCiphertext(t[b]) : std::move(tmp);
    }
    return aligned_.emplace(key, std::move(v)).first->second;
  }

  // T_i at level l for every (i, l) of `want` (not yet cached), all lanes, in shared launches
  // (AtLevelBatch: the scaled copies side by side, one batched rescale per target level)
  void align_many(const std::vector<std::pair<int, size_t>>& want) {
    std::set<std::pair<int, size_t>> keys;
    for (const auto& w : want)
      if (lvl(get(w.first)) != w.second && !aligned_.count(w)) keys.insert(w);
    if (keys.empty()) return;
    std::vector<const PhantomCiphertext*> src;
    std::vector<size_t> tgt;
    for (const auto& [i, l] : keys)
      for (size_t b = 0; b < B; ++b) {
        src.push_back(&get(i)[b]);
        tgt.push_back(l);
      }
    std::vector<PhantomCiphertext> r = AtLevelBatch(cc, src, tgt, sf);
    size_t k = 0;
    for (const auto& key : keys) {
      Lanes v(B);
      for (size_t b = 0; b < B; ++b, ++k) v[b] = r[k].size() ? std::move(r[k]) : PhantomCiphertext(get(key.first)[b]);
      aligned_.emplace(key, std::move(v));
    }
  }

  static int half_of(int i) {
    int a = 1;
    while (2 * a < i) a *= 2;  // a >= i / 2, a < i
    return a;
  }

  // T_i for every i of `idx` (absent so far, operands present or computable), all lanes, the
  // products in one batch: T_2a = 2 T_a^2 - 1 (doubling and constant folded in before the one
  // key switch); T_i = 2 T_a T_(i-a) - T_(2a-i), T_(2a-i) joining the product before its rescale
  // when it is not deeper than the product
  void compute(const std::vector<int>& idx) {
    for (int i : idx) {  // operands first (they may need a batch of their own)
      const int a = half_of(i);
      get(a);
      if (2 * a != i) {
        get(i - a);
        get(2 * a - i);
      }
    }
    std::vector<std::pair<int, size_t>> want;  // the operands' alignments, made together
    for (int i : idx) {
      const int a = half_of(i);
      if (2 * a == i) continue;
      const size_t l = std::max(lvl(get(a)), lvl(get(i - a)));
      want.push_back({a, l});
      want.push_back({i - a, l});
    }
    align_many(want);
    std::vector<MulAddJob> jobs;
    std::vector<std::pair<int, const Lanes*>> late;  // T_(2a-i) deeper than the product: subtracted after
    for (int i : idx) {
      const int a = half_of(i);
      if (2 * a == i) {
        const Lanes& ta = get(a);
        for (size_t b = 0; b < B; ++b) jobs.push_back(MulAddJob{&ta[b], &ta[b], 2, {}, -1.0});
        continue;
      }
      const size_t l = std::max(lvl(get(a)), lvl(get(i - a)));
      const Lanes& x = aligned(a, l);
      const Lanes& y = aligned(i - a, l);
      const Lanes& z = get(2 * a - i);
      const bool fold = lvl(z) <= l;
      for (size_t b = 0; b < B; ++b) {
        MulAddJob j{&x[b], &y[b], 2, {}, 0.0};
        if (fold) j.terms.push_back({&z[b], -1.0});
        jobs.push_back(std::move(j));
      }
      if (!fold) late.push_back({i, &z});
    }
    // products of one level share a batch (a generation's members always do)
    std::map<size_t, std::vector<size_t>> by_level;
    for (size_t k = 0; k < jobs.size(); ++k) by_level[level_of(*jobs[k].a)].push_back(k);
    std::vector<PhantomCiphertext> out(jobs.size());
    for (auto& [l, ks] : by_level) {
      std::vector<MulAddJob> part;
      for (size_t k : ks) part.push_back(jobs[k]);
      std::vector<PhantomCiphertext> r = MulAddRescaleBatch(cc, part, rlk);
      for (size_t m = 0; m < ks.size(); ++m) out[ks[m]] = std::move(r[m]);
    }
    for (size_t m = 0; m < idx.size(); ++m) {
      Lanes v(B);
      for (size_t b = 0; b < B; ++b) v[b] = std::move(out[m * B + b]);
      T.emplace(idx[m], std::move(v));
    }
    for (auto& [i, z] : late)
      for (size_t b = 0; b < B; ++b) EvalSubAutoInplace(cc, T.at(i)[b], (*z)[b], sf);
  }

  const Lanes& get(int i) {
    auto it = T.find(i);
    if (it != T.end()) return it->second;
    compute({i});
    return T.at(i);
  }

  // ---- the series as a tree: p = q T_m + r down to degree <= kLeafDegree leaves ----------
  struct Node {
    std::vector<double> c;  // leaf coefficients
    int m = 0;              // inner node: q T_m + r
    std::unique_ptr<Node> q, r;
    Lanes v;                // a leaf's value
  };

  static std::unique_ptr<Node> plan(const std::vector<double>& c) {
    auto node = std::make_unique<Node>();
    int d = static_cast<int>(c.size()) - 1;
    if (d <= kLeafDegree) {
      node->c = c;
      while (d > 0 && node->c[d] == 0.0) --d;
      node->c.resize(d + 1);
      return node;
    }
    const int m = cheb_split(d);
    // c_i T_i = c_i (2 T_m T_(i-m) - T_(2m-i)) for m < i <= d (<= 2m); i = m gives T_m T_0
    std::vector<double> q(d - m + 1, 0.0), r(c.begin(), c.begin() + m);
    q[0] = c[m];
    for (int i = m + 1; i <= d; ++i) {
      q[i - m] = 2.0 * c[i];
      r[2 * m - i] -= c[i];
    }
    node->m = m;
    node->q = plan(q);
    node->r = plan(r);
    return node;
  }

  static void collect(Node* n, std::vector<Node*>& out) {
    if (!n->m) {
      out.push_back(n);
      return;
    }
    collect(n->q.get(), out);
    collect(n->r.get(), out);
  }

  // every leaf sum_i c_i T_i lands on the deepest level of its T_1..T_d with scale sf[l]^2;
  // the leaves of one level are evaluated together by one kernel per lane that reads each T_i
  // once (FHECKKSRNS::leaf_tables caches the constant tables) into one buffer, and rescaled
  // together by one batched rescale into their own ciphertexts
  void eval_leaves(std::vector<Node*>& leaves) {
    std::map<size_t, std::vector<Node*>> by_level;
    for (Node* lf : leaves) {
      const int d = static_cast<int>(lf->c.size()) - 1;
      if (d < 1) continue;  // a constant remainder: its parent's product takes it as a constant
      size_t l = 0;
      for (int i = 1; i <= d; ++i) l = std::max(l, lvl(get(i)));
      by_level[l].push_back(lf);
    }
    const size_t n = cc.poly_degree();
    hipStream_t s = cc.stream();
    for (auto& [l, group] : by_level) {
      for (size_t g0 = 0; g0 < group.size(); g0 += phx::kLeafMaxM) {
        const int M = static_cast<int>(std::min<size_t>(phx::kLeafMaxM, group.size() - g0));
        int K = 0;
        for (int m = 0; m < M; ++m) K = std::max(K, static_cast<int>(group[g0 + m]->c.size()) - 1);
        const size_t chain = l + 1, L = cc.get_context_data(chain).coeff_modulus_size();
        const double target = sf.at(l) * sf.at(l);
        std::vector<uint64_t> tab(2 * static_cast<size_t>(M) * K * L + static_cast<size_t>(M) * L, 0);
        uint64_t* cv = tab.data();
        uint64_t* cs = cv + static_cast<size_t>(M) * K * L;
        uint64_t* ca = cs + static_cast<size_t>(M) * K * L;
        for (int m = 0; m < M; ++m) {
          const std::vector<double>& c = group[g0 + m]->c;
          for (int k = 0; k < K; ++k) {
            const double coeff = k + 1 < static_cast<int>(c.size()) ? c[k + 1] : 0.0;
            const size_t off = (static_cast<size_t>(m) * K + k) * L;
            ScalarResidues(cc, chain, coeff * target / get(k + 1)[0].scale(), cv + off, cs + off);
          }
          ScalarResidues(cc, chain, c[0] * target, ca + static_cast<size_t>(m) * L, nullptr);
        }
        const uint64_t* coef = tables.get(tab, s);
        const size_t cts = static_cast<size_t>(M) * B, ct_words = 2 * L * n;
        DeviceBuffer<uint64_t> w(cts * ct_words, s);  // leaf (m, lane b) at ((m B + b) 2 L) n
        for (size_t b = 0; b < B; ++b) {
          phx::LeafArgs la;
          la.K = K;
          la.M = M;
          la.L = static_cast<int>(L);
          la.q = cc.mod_QP().q;
          la.barrett = cc.mod_QP().barrett;
          la.coef = coef;
          la.cadd = la.coef + 2 * static_cast<size_t>(M) * K * L;
          for (int k = 0; k < K; ++k) {
            la.in[k] = get(k + 1)[b].data();
            la.in_stride[k] = get(k + 1)[b].coeff_modulus_size() * n;
          }
          for (int m = 0; m < M; ++m) la.out[m] = w.get() + (static_cast<size_t>(m) * B + b) * ct_words;
          hip_ok(phx::leaf_combine(la, n, s), "Chebyshev leaves");
        }
        // scale target / q_last, degree 1 (EvalModReduceInPlace of a degree-2 leaf)
        const RnsTool& rt = cc.get_context_data(chain).gpu_rns_tool();
        const double qlast = static_cast<double>(rt.base_Ql().back());
        std::vector<uint64_t*> outs(cts);
        for (int m = 0; m < M; ++m) {
          Lanes& v = group[g0 + m]->v;
          v.assign(B, PhantomCiphertext());
          for (size_t b = 0; b < B; ++b) {
            v[b].resize(cc, chain + 1, 2, s, false);
            v[b].set_ntt_form(true);
            v[b].set_scale(target / qlast);
            v[b].SetNoiseScaleDeg(1);
            outs[static_cast<size_t>(m) * B + b] = v[b].data();
          }
        }
        for (size_t c0 = 0; c0 < cts; c0 += phx::kMaxKsProds)
          rt.rescale_ntt_to(w.get() + c0 * ct_words, outs.data() + c0,
                            std::min<size_t>(phx::kMaxKsProds, cts - c0), cc.gpu_rns_tables(), s);
      }
    }
  }

  static bool has_value(const Node* nd) { return nd->m || nd->c.size() > 1; }

  // the products q T_m + r of every node in `nodes` (their children evaluated), one batched key
  // switch per product level: r joins a product before its rescale when it is not deeper than it,
  // a constant r as the product's constant
  void combine_round(const std::vector<Node*>& nodes) {
    std::deque<PhantomCiphertext> tmp;  // AtLevel copies, alive through the batch
    std::vector<MulAddJob> jobs;
    std::vector<std::pair<Node*, size_t>> dst;
    std::vector<Node*> late;  // r deeper than the product: added after the rescale
    // every operand's alignment first, in shared launches: T_m (cached) and the q values
    std::vector<std::pair<int, size_t>> want;
    std::vector<const PhantomCiphertext*> qsrc;
    std::vector<size_t> qtgt;
    for (Node* nd : nodes) {
      const size_t l = std::max(lvl(nd->q->v), lvl(get(nd->m)));
      want.push_back({nd->m, l});
      for (size_t b = 0; b < B; ++b) {
        qsrc.push_back(&nd->q->v[b]);
        qtgt.push_back(l);
      }
    }
    align_many(want);
    std::vector<PhantomCiphertext> qal = AtLevelBatch(cc, qsrc, qtgt, sf);
    size_t qk = 0;
    for (Node* nd : nodes) {
      const Lanes& qv = nd->q->v;
      const Node* rn = nd->r.get();
      const size_t l = std::max(lvl(qv), lvl(get(nd->m)));
      const Lanes& y = aligned(nd->m, l);
      const bool rv = has_value(rn), fold = rv && lvl(rn->v) <= l;
      for (size_t b = 0; b < B; ++b, ++qk) {
        tmp.emplace_back(std::move(qal[qk]));
        const PhantomCiphertext& x = tmp.back().size() ? tmp.back() : qv[b];
        MulAddJob j{&x, &y[b], 1, {}, 0.0};
        if (!rv) j.constant = rn->c.empty() ? 0.0 : rn->c[0];
        if (fold) j.terms.push_back({&rn->v[b], 1.0});
        jobs.push_back(std::move(j));
        dst.push_back({nd, b});
      }
      if (rv && !fold) late.push_back(nd);
      nd->v.assign(B, PhantomCiphertext());
    }
    std::map<size_t, std::vector<size_t>> by_level;
    for (size_t k = 0; k < jobs.size(); ++k) by_level[level_of(*jobs[k].a)].push_back(k);
    for (auto& [l, ks] : by_level) {
      std::vector<MulAddJob> part;
      for (size_t k : ks) part.push_back(jobs[k]);
      std::vector<PhantomCiphertext> r = MulAddRescaleBatch(cc, part, rlk);
      for (size_t m = 0; m < ks.size(); ++m) dst[ks[m]].first->v[dst[ks[m]].second] = std::move(r[m]);
    }
    for (Node* nd : late)
      for (size_t b = 0; b < B; ++b) EvalAddAutoInplace(cc, nd->v[b], nd->r->v[b], sf);
    for (Node* nd : nodes) {  // the children's values are consumed
      nd->q->v.clear();
      nd->r->v.clear();
    }
  }

  static int height(Node* nd, std::map<int, std::vector<Node*>>& by_h) {
    if (!nd->m) return 0;
    const int h = 1 + std::max(height(nd->q.get(), by_h), height(nd->r.get(), by_h));
    by_h[h].push_back(nd);
    return h;
  }

  // every T_i the tree reads: the leaves' T_1 .. T_d and the split points T_m
  static void needed(const Node* nd, std::set<int>& need) {
    if (!nd->m) {
      for (int i = 1; i < static_cast<int>(nd->c.size()); ++i) need.insert(i);
      return;
    }
    need.insert(nd->m);
    needed(nd->q.get(), need);
    needed(nd->r.get(), need);
  }

  Lanes eval(const std::vector<double>& c) {
    std::unique_ptr<Node> root = plan(c);
    std::set<int> need;
    needed(root.get(), need);
    ladder(need);
    std::vector<Node*> leaves;
    collect(root.get(), leaves);
    eval_leaves(leaves);
    std::map<int, std::vector<Node*>> by_h;
    height(root.get(), by_h);
    for (auto& [h, nodes] : by_h) combine_round(nodes);  // bottom-up, one round per height
    return std::move(root->v);
  }

  // the needed T_i (and what they are built from) generation by generation: T_(2^(g-1)+1) ..
  // T_(2^g) depend only on earlier generations and share a level, so each generation is one
  // batched key switch (T_16 joins T_9 .. T_15)
  void ladder(const std::set<int>& need) {
    std::set<int> all;
    std::vector<int> stack(need.begin(), need.end());
    while (!stack.empty()) {
      const int i = stack.back();
      stack.pop_back();
      if (i < 2 || !all.insert(i).second) continue;
      const int a = half_of(i);
      stack.push_back(a);
      if (2 * a != i) {
        stack.push_back(i - a);
        stack.push_back(2 * a - i);
      }
    }
    for (int lo = 2, hi = 2; !all.empty() && lo <= *all.rbegin(); lo = hi + 1, hi *= 2) {
      std::vector<int> members;
      for (int i : all)
        if (i >= lo && i <= hi && !T.count(i)) members.push_back(i);
      if (!members.empty()) compute(members);
    }
  }
};

}  // namespace

// ======================================================================================
// FHECKKSRNS
// ======================================================================================

const uint64_t* LeafTableCache::get(const std::vector<uint64_t>& table, hipStream_t s) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = tables_.find(table);
  if (it == tables_.end()) {
    DeviceBuffer<uint64_t> d;
    d.upload(table, s);  // once per distinct table: the same constants recur every bootstrap
    it = tables_.emplace(table, std::move(d)).first;
  }
  return it->second.get();
}

FHECKKSRNS::FHECKKSRNS(PhantomCKKSEncoder& encoder) : encoder_(encoder) {}

// GetDepthByDegree (src/util.cu:44-71): the reference's Paterson-Stockmeyer depth of a degree-d
// Chebyshev series, its affine map included
static uint32_t reference_series_depth(int d) { return ps::GetDepthByDegree(static_cast<size_t>(d)); }

uint32_t FHECKKSRNS::GetBootstrapDepth(const std::vector<uint32_t>& levelBudget) {
  return levelBudget.at(0) + levelBudget.at(1) + reference_series_depth(kChebDegree) + R_UNIFORM;
}

uint32_t FHECKKSRNS::GetBootstrapDepthTight(const std::vector<uint32_t>& levelBudget) {
  return levelBudget.at(0) + levelBudget.at(1) + static_cast<uint32_t>(cheb_depth(kChebDegree)) + R_UNIFORM;
}

void FHECKKSRNS::build_levels(const PhantomContext& cc, bool encode_dir, const LevelArgs& args, uint32_t slots,
                              std::vector<LTLevel>& out, bool encode) const {
  const std::vector<int>& sizes = args.sizes;
  const double constant = args.constant;
  const size_t first_chain = args.first_chain;
  const uint32_t dim1 = args.dim1;
  const size_t n = cc.poly_degree() / 2;  // slots of the ring
  const size_t ns = slots;                // slots of the (sub)problem: n = full packing
  const int logslots = arith::log2_exact(ns);
  std::vector<int> order;
  for (int s = 1; s <= logslots; ++s) order.push_back(s);
  if (encode_dir) std::reverse(order.begin(), order.end());
  // sparse packing (ns < n): the ns-slot maps act on every ns-block of the ring's slots.  The
  // CoeffToSlot output w = c_lo + i c_hi (ns-periodic) is multiplied by 1 on even blocks and -i on
  // odd ones, so w + conj(w) holds [c_lo | c_hi] in 2 ns-periodic real slots; SlotToCoeff reads
  // them as [c_lo | i c_hi], and a final rotation by ns adds the two halves (EvalBootstrap).
  boot::cvec out_mask, in_mask;
  if (ns < n) {
    out_mask.assign(2 * ns, {1.0, 0.0});
    in_mask.assign(2 * ns, {1.0, 0.0});
    for (size_t p = ns; p < 2 * ns; ++p) {
      out_mask[p] = {0.0, -1.0};
      in_mask[p] = {0.0, 1.0};
    }
  }
  out.clear();
  size_t idx = 0;
  for (size_t gi = 0; gi < sizes.size(); ++gi) {
    boot::DiagMap T;
    T.emplace(0, boot::cvec(ns, {1.0, 0.0}));
    int s_min = logslots;
    for (int t = 0; t < sizes[gi]; ++t) {
      const int s = order[idx++];
      s_min = std::min(s_min, s);
      T = boot::compose(boot::stage(ns, s, encode_dir), T, ns);
    }
    const bool scale_here = encode_dir ? gi == 0 : gi + 1 == sizes.size();
    if (scale_here) {
      const std::complex<double> cf = args.times_i ? std::complex<double>(0.0, constant) : std::complex<double>(constant, 0.0);
      for (auto& kv : T)
        for (auto& x : kv.second) x *= cf;
    }
    if (ns < n) {
      const bool last_enc = encode_dir && gi + 1 == sizes.size();
      const bool first_dec = !encode_dir && gi == 0;
      T = boot::lift_blocks(T, ns, n, last_enc ? &out_mask : nullptr, first_dec ? &in_mask : nullptr);
    }
    LTLevel lv;
    lt_shape(lv, T, n, dim1, 1 << (s_min - 1));
    lv.chain = first_chain + gi;
    if (encode) encode_level(cc, lv, T);
    out.push_back(std::move(lv));
  }
}

void FHECKKSRNS::lt_shape(LTLevel& lv, const boot::DiagMap& T, size_t n, uint32_t dim1, int stride) {
  lv.stride = stride;
  int kmin = 0, kmax = 0;
  for (const auto& kv : T) {
    int a = kv.first;
    if (a > static_cast<int>(n / 2)) a -= static_cast<int>(n);
    if (a % lv.stride) throw std::logic_error("diagonal offset not a multiple of the stride");
    kmin = std::min(kmin, a / lv.stride);
    kmax = std::max(kmax, a / lv.stride);
  }
  lv.center = -kmin;
  lv.D = kmax - kmin + 1;
  lv.g = 1;
  if (dim1) {
    if (dim1 & (dim1 - 1)) throw std::invalid_argument("dim1 must be a power of two");
    lv.g = static_cast<int>(std::min<uint32_t>(dim1, static_cast<uint32_t>(phx::kLtMaxG)));
  } else {
    // g^2 >= 2 D: twice the baby steps of the square split.  A hoisted baby step is one fused
    // key switch + automorphism; a giant step is a moddown + modup (one INTT over Ql u P and an
    // NTT over every digit) before its key switch, so fewer giant steps pay: 256 diagonals as
    // g 32 x b 8 instead of 16 x 16 take the bootstrap from 29.7 to 27.9 ms
    // (profiles/r02/lt_baby_giant_split.txt); PHX_LT_SQUARE=1 restores the square split.
    static const bool square = std::getenv("PHX_LT_SQUARE") != nullptr;
    while (lv.g * lv.g < (square ? 1 : 2) * lv.D && lv.g < phx::kLtMaxG) lv.g *= 2;
  }
  lv.b = (lv.D + lv.g - 1) / lv.g;
  if (lv.g > phx::kLtMaxG || lv.b > phx::kLtMaxB) throw std::invalid_argument("linear transform level too large");
}

void FHECKKSRNS::encode_level(const PhantomContext& cc, LTLevel& lv, const boot::DiagMap& T) const {
  const size_t n = cc.poly_degree() / 2;
  const double scale = sf_.at(lv.chain - 1);
  lv.pts.clear();
  lv.pts.resize(lv.D);
  // the level's diagonals: their host encodings (FFT + exact RNS rounding) run on host threads,
  // a chunk at a time, each chunk's uploads + NTTs queued on the stream behind it
  std::vector<std::pair<int, const boot::cvec*>> jobs;
  for (int u = 0; u < lv.D; ++u) {
    const long off = static_cast<long>(u - lv.center) * lv.stride;
    const int key = static_cast<int>(((off % static_cast<long>(n)) + static_cast<long>(n)) % static_cast<long>(n));
    auto it = T.find(key);
    if (it != T.end()) jobs.emplace_back(u, &it->second);
  }
  const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<std::vector<uint64_t>> host(nt);
  for (size_t c0 = 0; c0 < jobs.size(); c0 += nt) {
    const size_t cnt = std::min<size_t>(nt, jobs.size() - c0);
    auto work = [&](size_t w) {
      const int u = jobs[c0 + w].first;
      const boot::cvec& diag = *jobs[c0 + w].second;
      // pre-rotate by -(g i stride) so the giant rotation can follow the inner sum
      const size_t sh = static_cast<size_t>((u / lv.g) * lv.g) * lv.stride % n;
      boot::cvec rot(n);
      for (size_t p = 0; p < n; ++p) rot[p] = diag[(p + n - sh) % n];
      encoder_.encode_ext_host(cc, rot, scale, lv.chain, host[w], 1);
    };
    std::vector<std::thread> th;
    for (size_t w = 1; w < cnt; ++w) th.emplace_back(work, w);
    work(0);
    for (auto& t : th) t.join();
    for (size_t w = 0; w < cnt; ++w) {
      auto pt = std::make_unique<PhantomPlaintext>();
      encoder_.upload_ext_async(cc, host[w], scale, *pt, lv.chain);
      lv.pts[jobs[c0 + w].first] = std::move(pt);
    }
    PHX_CHECK(hipStreamSynchronize(cc.stream()));  // host[] is rewritten by the next chunk
  }
  std::vector<std::shared_ptr<PhantomPlaintext>> view;  // (attach reads the pointers only)
  attach(cc, lv, view);
}

// the device pointer table [b][g] of a level's plaintexts (lv.pts when `ext` is empty, else the
// caller's set); absent diagonals read a zero plaintext
void FHECKKSRNS::attach(const PhantomContext& cc, LTLevel& lv,
                        const std::vector<std::shared_ptr<PhantomPlaintext>>& ext) const {
  std::vector<const uint64_t*> ptrs(static_cast<size_t>(lv.b) * lv.g, nullptr);
  for (size_t u = 0; u < ptrs.size(); ++u) {
    const PhantomPlaintext* p = nullptr;
    if (u < static_cast<size_t>(lv.D)) p = ext.empty() ? lv.pts[u].get() : ext[u].get();
    if (p) {
      ptrs[u] = p->data();
      continue;
    }
    if (!lv.zero) {
      const size_t limbs = cc.get_context_data(lv.chain).coeff_modulus_size() + cc.size_P();
      lv.zero.allocate(limbs * cc.poly_degree(), cc.stream());
      PHX_CHECK(hipMemsetAsync(lv.zero.get(), 0, limbs * cc.poly_degree() * sizeof(uint64_t), cc.stream()));
    }
    ptrs[u] = lv.zero.get();
  }
  lv.d_pts.upload(ptrs, cc.stream());
}

void FHECKKSRNS::EvalBootstrapSetup(const PhantomContext& cc, const std::vector<uint32_t>& levelBudget, double scale,
                                    const std::vector<double>& sf, uint32_t correctionFactor, uint32_t slots_in,
                                    const std::vector<uint32_t>& dim1) {
  (void)scale;
  sf_big_.assign(sf.empty() ? 0 : sf.size() - 1, 0.0);
  for (size_t k = 0; k < sf_big_.size(); ++k) sf_big_[k] = sf[k] * sf[k];
  setup(cc, levelBudget, sf, correctionFactor, slots_in, dim1, true);
}

void FHECKKSRNS::EvalBootstrapSetup(const PhantomContext& cc, const std::vector<uint32_t>& levelBudget, double scale,
                                    const std::vector<double>& sf, const std::vector<double>& sf_big,
                                    const std::vector<uint32_t>& dim1, uint32_t slots, uint32_t correctionFactor,
                                    bool precompute) {
  (void)scale;
  // FLEXIBLEAUTO: m_scalingFactorsRealBig[k] = m_scalingFactorsReal[k]^2 (ciphertext.h:357-365)
  if (sf.empty() || sf_big.size() + 1 != sf.size())
    throw std::invalid_argument("EvalBootstrapSetup: scalingFactorsRealBig must have one entry less than scalingFactorsReal");
  for (size_t k = 0; k < sf_big.size(); ++k) {
    const double want = sf[k] * sf[k];
    if (!(std::fabs(sf_big[k] - want) <= 1e-12 * want))
      throw std::invalid_argument("EvalBootstrapSetup: scalingFactorsRealBig[" + std::to_string(k) +
                                  "] is not scalingFactorsReal[" + std::to_string(k) + "]^2 (FLEXIBLEAUTO)");
  }
  sf_big_ = sf_big;
  setup(cc, levelBudget, sf, correctionFactor, slots, dim1, precompute);
}

bool FHECKKSRNS::precomputed(uint32_t numSlots) const {
  std::lock_guard<std::mutex> lk(precom_mu_);
  auto it = precom_.find(numSlots ? numSlots : static_cast<uint32_t>(encoder_.slot_count()));
  return it != precom_.end() && it->second.encoded;
}

void FHECKKSRNS::setup(const PhantomContext& cc, const std::vector<uint32_t>& levelBudget,
                       const std::vector<double>& sf, uint32_t correctionFactor, uint32_t slots_in,
                       const std::vector<uint32_t>& dim1, bool precompute) {
  sf_ = sf;
  budget_ = levelBudget;
  const size_t N = cc.poly_degree();
  const uint32_t slots = slots_in ? slots_in : static_cast<uint32_t>(N / 2);
  if (slots > N / 2 || (slots & (slots - 1)) || slots < 2)
    throw std::invalid_argument("the number of slots must be a power of two between 2 and N/2");
  const int logslots = arith::log2_exact(slots);
  if (correctionFactor == 0) {
    const double tmp = std::round(-0.265 * (2 * std::log2(static_cast<double>(N)) + std::log2(static_cast<double>(slots))) + 19.1);
    correction_ = static_cast<uint32_t>(std::clamp(tmp, 7.0, 13.0));
  } else {
    correction_ = correctionFactor;
  }
  auto split = [&](uint32_t budget) {
    budget = std::clamp<uint32_t>(budget, 1, static_cast<uint32_t>(logslots));
    std::vector<int> sz(budget, logslots / static_cast<int>(budget));
    for (int i = 0; i < logslots % static_cast<int>(budget); ++i) ++sz[i];
    return sz;
  };
  const double q0 = static_cast<double>(cc.key_moduli()[0]);
  const std::vector<int> enc_sizes = split(levelBudget.at(0));
  std::vector<int> dec_sizes = split(levelBudget.at(1));
  std::reverse(dec_sizes.begin(), dec_sizes.end());
  const size_t depth_enc = enc_sizes.size(), depth_dec = dec_sizes.size();
  const size_t depth_mod = static_cast<size_t>(cheb_depth(kChebDegree)) + R_UNIFORM;
  // reference layout: the raise lands on the level the reference's extra Chebyshev level would
  // have consumed, so the output chain index is the reference's
  const size_t own = depth_enc + depth_mod + depth_dec;
  const size_t ref = depth_enc + depth_dec + reference_series_depth(kChebDegree) + R_UNIFORM;
  raise_level_ = tight_levels_ || ref < own ? 0 : ref - own;
  if (1 + raise_level_ + own > cc.size_Q())
    throw std::invalid_argument("not enough levels in the modulus chain for bootstrapping");
  // the sparse partial sum multiplies the coefficients it keeps by N / (2 slots)
  const double gap = static_cast<double>(N / 2) / slots;
  Precom pc;
  pc.slots = slots;
  // CoeffToSlot: slots become (t_lo + i t_hi) / (2 q0 K) (the conjugate split doubles them)
  const double s_raise = sf_.at(raise_level_);
  pc.enc_args = {enc_sizes, s_raise / (2.0 * gap * q0 * K_UNIFORM), 1 + raise_level_, dim1.size() > 0 ? dim1[0] : 0};
  // SlotToCoeff: from (t0_lo + i t0_hi) / q0 back to the message at the raise scale
  pc.dec_args = {dec_sizes, q0 / s_raise, 1 + raise_level_ + depth_enc + depth_mod, dim1.size() > 1 ? dim1[1] : 0};
  pc.encoded = precompute;
  build_levels(cc, true, pc.enc_args, slots, pc.enc, precompute);
  build_levels(cc, false, pc.dec_args, slots, pc.dec, precompute);
  {
    std::lock_guard<std::mutex> lk(precom_mu_);
    precom_[slots] = std::move(pc);
  }
  const double args[2] = {static_cast<double>(K_UNIFORM), static_cast<double>(R_UNIFORM)};
  cheb_ = boot::chebyshev_coefficients(boot::scaled_cosine, args, kChebDegree);
}

const FHECKKSRNS::Precom& FHECKKSRNS::precom(uint32_t numSlots, const PhantomContext& cc) const {
  const uint32_t slots = numSlots ? numSlots : static_cast<uint32_t>(cc.poly_degree() / 2);
  std::lock_guard<std::mutex> lk(precom_mu_);
  auto it = precom_.find(slots);
  if (it == precom_.end())
    throw std::invalid_argument("Precomputations for " + std::to_string(slots) +
                                " slots were not generated: call EvalBootstrapSetup and then EvalBootstrapKeyGen");
  Precom& pc = const_cast<Precom&>(it->second);
  if (!pc.encoded) {
    // deferred (precompute = false): encode the plaintexts of the same level structure now, once
    // (a std::map node is stable, and concurrent callers wait on precom_mu_)
    std::vector<LTLevel> enc, dec;
    build_levels(cc, true, pc.enc_args, slots, enc, true);
    build_levels(cc, false, pc.dec_args, slots, dec, true);
    pc.enc = std::move(enc);
    pc.dec = std::move(dec);
    pc.encoded = true;
  }
  return pc;
}

size_t FHECKKSRNS::OutputChainIndex(const std::vector<uint32_t>& levelBudget, uint32_t log_slots,
                                    uint32_t numIterations, bool tight) {
  if (log_slots < 1) throw std::invalid_argument("bad slot count");
  const size_t enc = std::clamp<uint32_t>(levelBudget.at(0), 1, log_slots);
  const size_t dec = std::clamp<uint32_t>(levelBudget.at(1), 1, log_slots);
  const size_t own_mod = static_cast<size_t>(cheb_depth(kChebDegree)) + R_UNIFORM;
  const size_t ref_mod = reference_series_depth(kChebDegree) + R_UNIFORM;
  const size_t raise = tight || ref_mod < own_mod ? 0 : ref_mod - own_mod;
  return 1 + raise + enc + own_mod + dec + (numIterations > 1 ? 1 : 0);
}

size_t FHECKKSRNS::output_chain_index(uint32_t numSlots, uint32_t numIterations) const {
  const uint32_t slots = numSlots ? numSlots : static_cast<uint32_t>(encoder_.slot_count());
  std::lock_guard<std::mutex> lk(precom_mu_);  // a deferred encoding may be reassigning pc.dec
  auto it = precom_.find(slots);
  if (it == precom_.end() || it->second.dec.empty()) throw std::invalid_argument("bootstrap setup missing");
  return it->second.dec.back().chain + 1 + (numIterations > 1 ? 1 : 0);
}

std::vector<int> FHECKKSRNS::rotation_indices(uint32_t numSlots) const {
  std::vector<int> r;
  const int n = static_cast<int>(encoder_.slot_count());
  auto add = [&](long x) {
    const int v = static_cast<int>(((x % n) + n) % n);
    if (v != 0 && std::find(r.begin(), r.end(), v) == r.end()) r.push_back(v);
  };
  const uint32_t slots = numSlots ? numSlots : static_cast<uint32_t>(n);
  std::lock_guard<std::mutex> lk(precom_mu_);
  auto it = precom_.find(slots);
  if (it == precom_.end()) throw std::invalid_argument("bootstrap setup missing for this slot count");
  for (const auto* lvs : {&it->second.enc, &it->second.dec})
    for (const LTLevel& lv : *lvs) {
      for (int j = 0; j < lv.g; ++j) add(static_cast<long>(j - lv.center) * lv.stride);
      for (int i = 1; i < lv.b; ++i) add(static_cast<long>(lv.g) * i * lv.stride);
    }
  // sparse packing: the partial sums before CoeffToSlot and the block fold after SlotToCoeff
  for (long j = 1; j * static_cast<long>(slots) < n; j <<= 1) add(j * static_cast<long>(slots));
  return r;
}

void FHECKKSRNS::claim_galois_keys(const PhantomSecretKey& sk) {
  uint64_t h = 0xcbf29ce484222325ull;  // FNV-1a over the secret's coefficients
  for (int8_t c : sk.coefficients()) h = (h ^ static_cast<uint8_t>(c)) * 0x100000001b3ull;
  if (h != galois_owner_) galois_keys_ = PhantomGaloisKey{};
  galois_owner_ = h;
}

void FHECKKSRNS::EvalBootstrapKeyGen(PhantomSecretKey& sk, const PhantomContext& cc, uint32_t numSlots) {
  claim_galois_keys(sk);
  std::vector<uint32_t> elts;
  for (int r : rotation_indices(numSlots)) elts.push_back(FindAutomorphismIndex2nComplex(r, cc.poly_degree()));
  elts.push_back(static_cast<uint32_t>(2 * cc.poly_degree() - 1));  // conjugation
  // keys of earlier setups (other slot counts) under the same secret stay; only the missing
  // elements are generated
  std::vector<uint32_t> need;
  for (uint32_t e : elts)
    if (!galois_keys_.has(e)) need.push_back(e);
  galois_keys_.merge(sk.create_galois_keys_fused(cc, need));
}

void FHECKKSRNS::EvalRotationKeyGen(PhantomSecretKey& sk, const PhantomContext& cc, const std::vector<int32_t>& indices) {
  claim_galois_keys(sk);
  std::vector<uint32_t> need;
  for (int32_t r : indices) {
    const uint32_t e = FindAutomorphismIndex2nComplex(r, cc.poly_degree());
    if (e != 1 && !galois_keys_.has(e) && std::find(need.begin(), need.end(), e) == need.end()) need.push_back(e);
  }
  if (!need.empty()) galois_keys_.merge(sk.create_galois_keys_fused(cc, need));
}

void FHECKKSRNS::EvalMultKeyGen(PhantomSecretKey& sk, const PhantomContext& cc) { mul_key_ = sk.gen_relinkey(cc); }

const void* FHECKKSRNS::baby_table(const PhantomContext& cc, const LTLevel& lv, size_t QlP) const {
  static_assert(sizeof(phx::KsBatchEntry) % sizeof(uint64_t) == 0, "entry of whole words");
  const size_t n = cc.poly_degree();
  std::vector<phx::KsBatchEntry> e(lv.g);
  for (int j = 0; j < lv.g; ++j) {
    const long r = static_cast<long>(j - lv.center) * lv.stride;
    const long nn = static_cast<long>(n / 2);
    if (((r % nn) + nn) % nn != 0) {  // else the identity: P (c0, c1) (KeySwitchExt)
      const uint32_t elt = FindAutomorphismIndex2nComplex(static_cast<int>(r), n);
      e[j].evk = galois_keys_.get(elt).public_keys_ptr();
      e[j].perm = cc.galois_perm(elt);
      e[j].binv = cc.galois_block_inv(elt);
    }
    e[j].out_off = static_cast<int64_t>(j * 2 * QlP * n);
  }
  const uint64_t* w = reinterpret_cast<const uint64_t*>(e.data());
  std::vector<uint64_t> words(w, w + e.size() * sizeof(phx::KsBatchEntry) / sizeof(uint64_t));
  std::lock_guard<std::mutex> lk(baby_mu_);
  auto& t = baby_tables_[&lv];
  if (t.first != words) {
    t.second.upload(words, cc.stream());
    t.first = std::move(words);
  }
  return t.second.get();
}

// one linear-transform level in three stages (apply_level runs them for one ciphertext,
// apply_level_pair for two with the inner products of both in one launch)
struct LevelWork {
  PhantomCiphertext tmp;
  const PhantomCiphertext* ct = nullptr;
  size_t Ql = 0, QlP = 0;
  DeviceBuffer<uint64_t> digits, babies, giants;
  phx::KsRotateBatchArgs ba;  // the baby steps' launch (level_babies with launch = false leaves it)
  PhantomCiphertext acc;
};

void FHECKKSRNS::level_babies(const PhantomContext& cc, const PhantomCiphertext& in, const LTLevel& lv,
                              LevelWork& w, bool launch, bool alloc_babies) const {
  w.ct = &AtLevel(cc, in, lv.chain - 1, sf_, w.tmp);
  const PhantomCiphertext& ct = *w.ct;
  const size_t n = cc.poly_degree(), Ql = cc.get_context_data(ct.chain_index()).coeff_modulus_size();
  const size_t QlP = Ql + cc.size_P();
  w.Ql = Ql;
  w.QlP = QlP;
  hipStream_t s = cc.stream();
  w.digits = EvalFastRotationPrecompute(cc, ct);
  // every baby step in one launch (keyswitch_rotate_batch): the digits and c0 are read from HBM
  // once for the level, not once per rotation; baby j at babies + j 2 QlP n
  const size_t baby_words = 2 * QlP * n;
  if (alloc_babies) w.babies = DeviceBuffer<uint64_t>(static_cast<size_t>(lv.g) * baby_words, s);
  const RnsTool& rt = cc.get_context_data(ct.chain_index()).gpu_rns_tool();
  phx::KsRotateBatchArgs& ba = w.ba;
  ba.digits = w.digits.get();
  ba.entries = static_cast<const phx::KsBatchEntry*>(baby_table(cc, lv, QlP));
  ba.count = static_cast<uint32_t>(lv.g);
  ba.qp = cc.mod_QP().q;
  ba.qp_barrett = cc.mod_QP().barrett;
  ba.ct = ct.data();
  ba.pmod = rt.bigP_mod_q();
  ba.pmod_shoup = rt.bigP_mod_q_shoup();
  ba.out = w.babies.get();
  ba.ql = static_cast<uint32_t>(Ql);
  ba.qlp = static_cast<uint32_t>(QlP);
  ba.size_q = static_cast<uint32_t>(cc.size_Q());
  ba.size_p = static_cast<uint32_t>(cc.size_P());
  ba.beta = static_cast<uint32_t>(rt.beta());
  ba.q60 = below_2_60(cc.key_moduli());
  if (launch) {
    hip_ok(phx::keyswitch_rotate_batch(ba, n, s), "linear transform baby steps");
    w.digits.release();
  }
  static const bool shapes = std::getenv("PHX_BOOT_TRACE") != nullptr;
  if (shapes)
    std::fprintf(stderr, "[lt] chain %zu Ql %zu beta %zu D %d g %d b %d\n", lv.chain, Ql, rt.beta(), lv.D, lv.g, lv.b);
  size_t rotations = 0;
  for (int j = 0; j < lv.g; ++j) {
    const long r = static_cast<long>(j - lv.center) * lv.stride, nn = static_cast<long>(n / 2);
    rotations += ((r % nn) + nn) % nn != 0;
  }
  traffic::keys(traffic::limb_bytes(rt.beta() * 2 * QlP * rotations, n));
  // the digits and c0 read, the baby steps written (not in the fused form)
  traffic::ciphertexts(
      traffic::limb_bytes(rt.beta() * QlP + Ql + (alloc_babies ? 2 * QlP * static_cast<size_t>(lv.g) : 0), n));
  // giant 0's inner sum goes straight into the accumulator, giants 1 .. b-1 into one buffer
  // [b - 1][2][QlP][n] so that their moddowns batch
  w.acc.resize(2, QlP, n, s, false);
  w.acc.set_chain_index(ct.chain_index());
  w.acc.set_ntt_form(true);
  w.giants = DeviceBuffer<uint64_t>(std::max<size_t>(static_cast<size_t>(lv.b - 1), 1) * 2 * QlP * n, s);
}

phx::LtArgs FHECKKSRNS::level_lt_args(const PhantomContext& cc, const LTLevel& lv, LevelWork& w) const {
  const size_t n = cc.poly_degree(), baby_words = 2 * w.QlP * n, ext_words = 2 * w.QlP * n;
  phx::LtArgs la;
  la.g = lv.g;
  la.b = lv.b;
  la.Ql = static_cast<int>(w.Ql);
  la.P = static_cast<int>(cc.size_P());
  la.size_Q = static_cast<int>(cc.size_Q());
  la.pts = lv.d_pts.get();
  la.q = cc.mod_QP().q;
  la.barrett = cc.mod_QP().barrett;
  la.q60 = below_2_60(cc.key_moduli());
  for (int j = 0; j < lv.g; ++j) la.baby[j] = w.babies.get() + static_cast<size_t>(j) * baby_words;
  la.out[0] = w.acc.data();
  for (int i = 1; i < lv.b; ++i) la.out[i] = w.giants.get() + static_cast<size_t>(i - 1) * ext_words;
  // the level's non-zero diagonals read once; the baby steps read and the inner sums written
  // once; the input read once (by the modup) and the output written once (after the giant steps)
  size_t nz = 0;
  for (const auto& p : lv.pts) nz += p ? 1 : 0;
  traffic::plaintexts(traffic::limb_bytes(nz * w.QlP, n));
  traffic::ciphertexts(traffic::limb_bytes(2 * w.QlP * static_cast<size_t>(lv.g + lv.b), n));
  return la;
}

PhantomCiphertext FHECKKSRNS::level_giants(const PhantomContext& cc, const LTLevel& lv, LevelWork& w) const {
  const PhantomCiphertext& ct = *w.ct;
  const size_t n = cc.poly_degree(), QlP = w.QlP, Ql = w.Ql, ext_words = 2 * QlP * n;
  const size_t G = static_cast<size_t>(lv.b - 1);
  hipStream_t s = cc.stream();
  w.babies.release();
  if (G > 0) {
    // giant steps accumulate in the extended basis (one moddown at the end).  Their c1's come down
    // to Ql and into their modup digits in one batched pass (one launch per stage over all G,
    // instead of G chains of small launches on concurrent streams, which a single launch over
    // the same limbs beats: profiles/r03/giant_batch/), then each key switch + rotation adds into
    // acc in turn
    const RnsTool& rt = cc.get_context_data(ct.chain_index()).gpu_rns_tool();
    const size_t dwords = rt.beta() * QlP * n;
    DeviceBuffer<uint64_t> digits(G * dwords, s);
    rt.moddown_modup(digits.get(), w.giants.get() + QlP * n, cc.gpu_rns_tables(), s, G, ext_words);
    for (size_t i = 1; i <= G; ++i)
      EvalRotateExtAccumulateDigits(cc, ct.chain_index(), w.giants.get() + (i - 1) * ext_words,
                                    digits.get() + (i - 1) * dwords, galois_keys_,
                                    static_cast<int>(static_cast<long>(lv.g) * static_cast<long>(i) * lv.stride), w.acc);
  }
  w.acc.set_scale(ct.scale() * sf_.at(lv.chain - 1));
  w.acc.SetNoiseScaleDeg(2);
  // giant steps: each inner sum read once, the level's result written once
  traffic::ciphertexts(traffic::limb_bytes(2 * QlP * static_cast<size_t>(lv.b) + 2 * (Ql - 1), n));
  w.giants.release();
  return KeySwitchDownRescale(cc, w.acc);
}

PhantomCiphertext FHECKKSRNS::apply_level(const PhantomContext& cc, const PhantomCiphertext& in,
                                          const LTLevel& lv) const {
  LevelWork w;
  level_babies(cc, in, lv, w);
  hip_ok(phx::lt_bsgs(level_lt_args(cc, lv, w), cc.poly_degree(), cc.stream()), "linear transform inner products");
  return level_giants(cc, lv, w);
}

std::vector<PhantomCiphertext> FHECKKSRNS::apply_level_group(const PhantomContext& cc,
                                                             const std::vector<const PhantomCiphertext*>& in,
                                                             const LTLevel& lv) const {
  const int K = static_cast<int>(in.size());
  if (K < 2 || K > phx::kLtGroupMax || K > phx::kKsGroupMax)
    throw std::invalid_argument("apply_level_group: 2 to 8 ciphertexts");
  std::vector<LevelWork> w(K);
  for (int c = 0; c < K; ++c) level_babies(cc, *in[c], lv, w[c], false);
  phx::KsRotateBatchGroupArgs ka;
  ka.count = K;
  for (int c = 0; c < K; ++c) ka.a[c] = w[c].ba;
  hip_ok(phx::keyswitch_rotate_batch_group(ka, cc.poly_degree(), cc.stream()), "linear transform baby steps (group)");
  for (LevelWork& x : w) x.digits.release();
  bool same_ql = true;
  std::vector<phx::LtArgs> la(K);
  for (int c = 0; c < K; ++c) {
    la[c] = level_lt_args(cc, lv, w[c]);
    same_ql &= w[c].Ql == w[0].Ql;
  }
  if (lv.g == 32 && lv.b <= 8 && same_ql) {
    const size_t ext_words = 2 * w[0].QlP * cc.poly_degree();
    phx::LtGroupArgs ga;
    ga.pts = la[0].pts;
    ga.q = la[0].q;
    ga.barrett = la[0].barrett;
    ga.g = la[0].g;
    ga.b = la[0].b;
    ga.Ql = la[0].Ql;
    ga.P = la[0].P;
    ga.size_Q = la[0].size_Q;
    ga.q60 = la[0].q60;
    ga.count = K;
    ga.baby_stride = ext_words;  // (the babies and inner sums are [2][QlP][n] ciphertexts, back to back)
    ga.giant_stride = ext_words;
    for (int c = 0; c < K; ++c) {
      ga.baby0[c] = w[c].babies.get();
      ga.acc[c] = w[c].acc.data();
      ga.giant1[c] = w[c].giants.get();
    }
    hip_ok(phx::lt_bsgs_group(ga, cc.poly_degree(), cc.stream()), "linear transform inner products (group)");
  } else {
    for (int c = 0; c < K; ++c) hip_ok(phx::lt_bsgs(la[c], cc.poly_degree(), cc.stream()), "linear transform inner products");
  }
  return level_giants_group(cc, lv, w);
}

std::vector<PhantomCiphertext> FHECKKSRNS::level_giants_group(const PhantomContext& cc, const LTLevel& lv,
                                                              std::vector<LevelWork>& w) const {
  const size_t K = w.size(), n = cc.poly_degree(), QlP = w[0].QlP, Ql = w[0].Ql, ext_words = 2 * QlP * n;
  const size_t G = static_cast<size_t>(lv.b - 1);
  hipStream_t s = cc.stream();
  bool same = true;
  for (const LevelWork& x : w) same &= x.QlP == QlP && x.ct->chain_index() == w[0].ct->chain_index();
  if (!same) {
    std::vector<PhantomCiphertext> r;
    for (LevelWork& x : w) r.push_back(level_giants(cc, lv, x));
    return r;
  }
  for (LevelWork& x : w) x.babies.release();
  if (G > 0) {
    // as level_giants, with each giant rotation of the K ciphertexts in one launch that reads
    // its key about once (keyswitch_rotate_group)
    const RnsTool& rt = cc.get_context_data(w[0].ct->chain_index()).gpu_rns_tool();
    const size_t dwords = rt.beta() * QlP * n;
    std::vector<DeviceBuffer<uint64_t>> digits;
    for (LevelWork& x : w) {
      digits.emplace_back(G * dwords, s);
      rt.moddown_modup(digits.back().get(), x.giants.get() + QlP * n, cc.gpu_rns_tables(), s, G, ext_words);
    }
    for (size_t i = 1; i <= G; ++i) {
      const uint32_t elt = FindAutomorphismIndex2nComplex(
          static_cast<int>(static_cast<long>(lv.g) * static_cast<long>(i) * lv.stride), n);
      phx::KsRotateGroupArgs ga;
      ga.count = static_cast<int>(K);
      for (size_t c = 0; c < K; ++c) {
        phx::KsRotateArgs& g = ga.a[c];
        g.digits = digits[c].get() + (i - 1) * dwords;
        g.evk = galois_keys_.get(elt).public_keys_ptr();
        g.qp = cc.mod_QP().q;
        g.qp_barrett = cc.mod_QP().barrett;
        g.c0 = w[c].giants.get() + (i - 1) * ext_words;
        g.out = w[c].acc.data();
        g.perm = cc.galois_perm(elt);
        g.ql = static_cast<uint32_t>(Ql);
        g.qlp = static_cast<uint32_t>(QlP);
        g.size_q = static_cast<uint32_t>(cc.size_Q());
        g.size_p = static_cast<uint32_t>(cc.size_P());
        g.beta = static_cast<uint32_t>(rt.beta());
        g.accumulate = true;
      }
      hip_ok(phx::keyswitch_rotate_group(ga, 2, n, s), "giant step key switch + permute + accumulate (group)");
      traffic::keys(traffic::limb_bytes(rt.beta() * 2 * QlP, n));  // read once for the group
    }
  }
  std::vector<PhantomCiphertext> r;
  for (LevelWork& x : w) {
    x.acc.set_scale(x.ct->scale() * sf_.at(lv.chain - 1));
    x.acc.SetNoiseScaleDeg(2);
    traffic::ciphertexts(traffic::limb_bytes(2 * QlP * static_cast<size_t>(lv.b) + 2 * (Ql - 1), n));
    x.giants.release();
    r.push_back(KeySwitchDownRescale(cc, x.acc));
  }
  return r;
}

PhantomCiphertext FHECKKSRNS::EvalCoeffsToSlots(const PhantomCiphertext& ct, const PhantomContext& cc,
                                                uint32_t numSlots) const {
  const Precom& pc = precom(numSlots, cc);
  PhantomCiphertext r = apply_level(cc, ct, pc.enc.at(0));
  for (size_t i = 1; i < pc.enc.size(); ++i) r = apply_level(cc, r, pc.enc[i]);
  return r;
}

PhantomCiphertext FHECKKSRNS::EvalSlotsToCoeffs(const PhantomCiphertext& ct, const PhantomContext& cc,
                                                uint32_t numSlots) const {
  const Precom& pc = precom(numSlots, cc);
  PhantomCiphertext r = apply_level(cc, ct, pc.dec.at(0));
  for (size_t i = 1; i < pc.dec.size(); ++i) r = apply_level(cc, r, pc.dec[i]);
  return r;
}

// ---- the reference's precompute / evaluate / rotation-index surface ------------------------------

std::vector<int32_t> FHECKKSRNS::dir_rotations(uint32_t slots, uint32_t M, bool encode_dir) const {
  std::lock_guard<std::mutex> lk(precom_mu_);
  auto it = precom_.find(slots);
  if (it == precom_.end())
    throw std::invalid_argument("Precomputations for " + std::to_string(slots) +
                                " slots were not generated Need to call EvalBootstrapSetup to proceed");
  const long quarter = static_cast<long>(M / 4);
  std::vector<int32_t> r;
  auto reduce = [](long x, long m) { return static_cast<int32_t>(((x % m) + m) % m); };  // ReduceRotation
  for (const LTLevel& lv : encode_dir ? it->second.enc : it->second.dec) {
    for (int j = 0; j < lv.g; ++j) r.push_back(reduce(static_cast<long>(j - lv.center) * lv.stride, quarter));
    for (int i = 0; i < lv.b; ++i) r.push_back(reduce(static_cast<long>(lv.g) * i * lv.stride, quarter));
  }
  // sparse packing: the partial sums before CoeffToSlot, the fold after SlotToCoeff
  if (4 * static_cast<long>(slots) != static_cast<long>(M)) {
    if (encode_dir) {
      for (long j = 1; j * 4 * static_cast<long>(slots) < static_cast<long>(M); j <<= 1) r.push_back(static_cast<int32_t>(j * slots));
    } else {
      r.push_back(static_cast<int32_t>(slots));
    }
  }
  std::sort(r.begin(), r.end());
  r.erase(std::unique(r.begin(), r.end()), r.end());
  r.erase(std::remove(r.begin(), r.end(), 0), r.end());
  r.erase(std::remove(r.begin(), r.end(), static_cast<int32_t>(quarter)), r.end());
  return r;
}

std::vector<int32_t> FHECKKSRNS::FindCoeffsToSlotsRotationIndices(uint32_t slots, uint32_t M) const {
  return dir_rotations(slots, M, true);
}

std::vector<int32_t> FHECKKSRNS::FindSlotsToCoeffsRotationIndices(uint32_t slots, uint32_t M) const {
  return dir_rotations(slots, M, false);
}

std::vector<int32_t> FHECKKSRNS::FindBootstrapRotationIndices(uint32_t slots, uint32_t M) const {
  std::vector<int32_t> r = FindCoeffsToSlotsRotationIndices(slots, M);
  const std::vector<int32_t> d = FindSlotsToCoeffsRotationIndices(slots, M);
  r.insert(r.end(), d.begin(), d.end());
  std::sort(r.begin(), r.end());
  r.erase(std::unique(r.begin(), r.end()), r.end());
  return r;
}

// the dense transform's level: every diagonal offset 0 .. slots-1 (stride 1)
static uint32_t dense_g(uint32_t slots, uint32_t dim) {
  if (dim) return dim;
  uint32_t g = 1;
  while (g * g < slots && g < static_cast<uint32_t>(phx::kLtMaxG)) g *= 2;
  return g;
}

std::vector<int32_t> FHECKKSRNS::FindLinearTransformRotationIndices(uint32_t slots, uint32_t M, uint32_t dim) const {
  if (slots == 0 || slots > M / 4) throw std::invalid_argument("FindLinearTransformRotationIndices: bad slot count");
  const uint32_t g = dense_g(slots, dim), b = (slots + g - 1) / g;
  std::vector<int32_t> r;
  for (uint32_t j = 1; j < g; ++j) r.push_back(static_cast<int32_t>(j % slots));
  for (uint32_t i = 1; i < b; ++i) r.push_back(static_cast<int32_t>((g * i) % slots));
  std::sort(r.begin(), r.end());
  r.erase(std::unique(r.begin(), r.end()), r.end());
  r.erase(std::remove(r.begin(), r.end(), 0), r.end());
  return r;
}

std::vector<std::shared_ptr<PhantomPlaintext>> FHECKKSRNS::EvalLinearTransformPrecompute(
    const PhantomContext& cc, const std::vector<std::vector<std::complex<double>>>& A, double scale, uint32_t L) const {
  const size_t n = cc.poly_degree() / 2, slots = A.size();
  if (slots != n) throw std::invalid_argument("EvalLinearTransformPrecompute: A must be (N/2) x (N/2) (full packing)");
  for (const auto& row : A)
    if (row.size() != slots) throw std::invalid_argument("EvalLinearTransformPrecompute: A is not square");
  // diagonal k: d_k[p] = A[p][(p + k) mod slots] (ExtractShiftedDiagonal, util.cu:298-312)
  boot::DiagMap T;
  for (size_t k = 0; k < slots; ++k) {
    boot::cvec d(slots);
    bool nz = false;
    for (size_t p = 0; p < slots; ++p) {
      d[p] = A[p][(p + k) % slots] * scale;
      nz |= d[p] != std::complex<double>(0.0, 0.0);
    }
    if (nz) T.emplace(static_cast<int>(k), std::move(d));
  }
  LTLevel lv;
  lv.stride = 1;
  lv.center = 0;
  lv.D = static_cast<int>(slots);
  lv.g = static_cast<int>(dense_g(static_cast<uint32_t>(slots), 0));
  lv.b = (lv.D + lv.g - 1) / lv.g;
  if (lv.g > phx::kLtMaxG || lv.b > phx::kLtMaxB)
    throw std::invalid_argument("EvalLinearTransformPrecompute: more diagonals than one level evaluates (N <= 2^12)");
  lv.chain = 1 + L;
  if (lv.chain >= cc.total_parm_size()) throw std::invalid_argument("EvalLinearTransformPrecompute: L beyond the chain");
  encode_level(cc, lv, T);
  std::vector<std::shared_ptr<PhantomPlaintext>> out(lv.D);
  for (int u = 0; u < lv.D; ++u) out[u] = std::shared_ptr<PhantomPlaintext>(std::move(lv.pts[u]));
  return out;
}

std::vector<std::shared_ptr<PhantomPlaintext>> FHECKKSRNS::EvalLinearTransformPrecompute(
    const PhantomContext&, const std::vector<std::vector<std::complex<double>>>&,
    const std::vector<std::vector<std::complex<double>>>&, uint32_t, double, uint32_t) const {
  throw std::logic_error(
      "EvalLinearTransformPrecompute(A, B, orientation): the reference declares it (include/bootstrap.cuh:133-136) "
      "but defines no body; sparse packing runs through EvalCoeffsToSlots / EvalSlotsToCoeffs instead");
}

PhantomCiphertext FHECKKSRNS::EvalLinearTransform(const std::vector<std::shared_ptr<PhantomPlaintext>>& A,
                                                  const PhantomCiphertext& ct, const PhantomContext& cc) const {
  const size_t n = cc.poly_degree() / 2;
  if (A.size() != n) throw std::invalid_argument("EvalLinearTransform: expects EvalLinearTransformPrecompute's N/2 plaintexts");
  LTLevel lv;
  lv.stride = 1;
  lv.center = 0;
  lv.D = static_cast<int>(n);
  lv.g = static_cast<int>(dense_g(static_cast<uint32_t>(n), 0));
  lv.b = (lv.D + lv.g - 1) / lv.g;
  lv.chain = 0;
  for (const auto& p : A)
    if (p) lv.chain = p->chain_index();
  if (!lv.chain) throw std::invalid_argument("EvalLinearTransform: every diagonal is zero");
  attach(cc, lv, A);
  return apply_level(cc, ct, lv);
}

std::vector<std::vector<std::shared_ptr<PhantomPlaintext>>> FHECKKSRNS::precompute_dir(
    const PhantomContext& cc, bool encode_dir, const std::vector<std::complex<double>>& A,
    const std::vector<uint32_t>& rotGroup, bool flag_i, double scale, uint32_t L) const {
  const uint32_t slots = static_cast<uint32_t>(rotGroup.size());
  const uint64_t M = 2 * cc.poly_degree();
  // the roots this engine's factorisation uses (ksiPows and the powers of 5, bootstrap.cu:92-107)
  if (A.size() < M) throw std::invalid_argument("A must hold the 2N-th roots of unity (ksiPows)");
  for (uint64_t j = 0; j < M; ++j) {
    const double ang = 2.0 * M_PI * static_cast<double>(j) / static_cast<double>(M);
    if (std::abs(A[j] - std::complex<double>(std::cos(ang), std::sin(ang))) > 1e-9)
      throw std::invalid_argument("A[" + std::to_string(j) + "] is not exp(2 pi i j / 2N)");
  }
  uint64_t g5 = 1;
  for (uint32_t j = 0; j < slots; ++j, g5 = g5 * 5 % M)
    if (rotGroup[j] != g5) throw std::invalid_argument("rotGroup must be 5^j mod 2N");
  LevelArgs args;
  {
    std::lock_guard<std::mutex> lk(precom_mu_);
    auto it = precom_.find(slots);
    if (it == precom_.end())
      throw std::invalid_argument("Precomputations for " + std::to_string(slots) +
                                  " slots were not generated Need to call EvalBootstrapSetup to proceed");
    args = encode_dir ? it->second.enc_args : it->second.dec_args;
  }
  args.constant = scale;
  args.times_i = flag_i;
  // lEnc / lDec: the first level's chain, 1 + (size_Q - L - levelBudget) dropped towers (L = 0: chain 1)
  const size_t budget = args.sizes.size();
  if (L != 0 && static_cast<size_t>(L) + budget > cc.size_Q()) throw std::invalid_argument("L leaves too few levels");
  args.first_chain = L == 0 ? 1 : 1 + cc.size_Q() - L - budget;
  std::vector<LTLevel> levels;
  build_levels(cc, encode_dir, args, slots, levels, true);
  std::vector<std::vector<std::shared_ptr<PhantomPlaintext>>> out(levels.size());
  for (size_t gi = 0; gi < levels.size(); ++gi) {
    out[gi].resize(levels[gi].D);
    for (int u = 0; u < levels[gi].D; ++u) out[gi][u] = std::shared_ptr<PhantomPlaintext>(std::move(levels[gi].pts[u]));
  }
  return out;
}

PhantomCiphertext FHECKKSRNS::apply_dir(const std::vector<std::vector<std::shared_ptr<PhantomPlaintext>>>& A,
                                        const PhantomCiphertext& ct, const PhantomContext& cc, uint32_t numSlots,
                                        bool encode_dir) const {
  const uint32_t slots = numSlots ? numSlots : static_cast<uint32_t>(cc.poly_degree() / 2);
  LevelArgs args;
  {
    std::lock_guard<std::mutex> lk(precom_mu_);
    auto it = precom_.find(slots);
    if (it == precom_.end())
      throw std::invalid_argument("Precomputations for " + std::to_string(slots) +
                                  " slots were not generated Need to call EvalBootstrapSetup to proceed");
    args = encode_dir ? it->second.enc_args : it->second.dec_args;
  }
  std::vector<LTLevel> levels;
  build_levels(cc, encode_dir, args, slots, levels, false);  // the shape only
  if (A.size() != levels.size()) throw std::invalid_argument("plaintext set does not match the setup's level budget");
  PhantomCiphertext r;
  for (size_t gi = 0; gi < levels.size(); ++gi) {
    LTLevel& lv = levels[gi];
    if (A[gi].size() != static_cast<size_t>(lv.D)) throw std::invalid_argument("plaintext set does not match the setup");
    lv.chain = 0;
    for (const auto& p : A[gi])
      if (p) lv.chain = p->chain_index();
    if (!lv.chain) throw std::invalid_argument("a level of the plaintext set is empty");
    attach(cc, lv, A[gi]);
    r = apply_level(cc, gi ? r : ct, lv);
  }
  return r;
}

std::vector<std::vector<std::shared_ptr<PhantomPlaintext>>> FHECKKSRNS::EvalCoeffsToSlotsPrecompute(
    const PhantomContext& cc, const std::vector<std::complex<double>>& A, const std::vector<uint32_t>& rotGroup,
    const std::vector<double>& sf, bool flag_i, double scale, uint32_t L) const {
  if (!sf.empty() && sf.size() != sf_.size()) throw std::invalid_argument("scaling factors differ from the setup's");
  return precompute_dir(cc, true, A, rotGroup, flag_i, scale, L);
}

std::vector<std::vector<std::shared_ptr<PhantomPlaintext>>> FHECKKSRNS::EvalSlotsToCoeffsPrecompute(
    const PhantomContext& cc, const std::vector<std::complex<double>>& A, const std::vector<uint32_t>& rotGroup,
    const std::vector<double>& sf, bool flag_i, double scale, uint32_t L) const {
  if (!sf.empty() && sf.size() != sf_.size()) throw std::invalid_argument("scaling factors differ from the setup's");
  return precompute_dir(cc, false, A, rotGroup, flag_i, scale, L);
}

PhantomCiphertext FHECKKSRNS::EvalCoeffsToSlots(const std::vector<std::vector<std::shared_ptr<PhantomPlaintext>>>& A,
                                                const PhantomCiphertext& ctxt, const PhantomContext& cc,
                                                uint32_t numSlots) const {
  return apply_dir(A, ctxt, cc, numSlots, true);
}

PhantomCiphertext FHECKKSRNS::EvalSlotsToCoeffs(const std::vector<std::vector<std::shared_ptr<PhantomPlaintext>>>& A,
                                                const PhantomCiphertext& ctxt, const PhantomContext& cc,
                                                uint32_t numSlots) const {
  return apply_dir(A, ctxt, cc, numSlots, false);
}

PhantomCiphertext FHECKKSRNS::EvalChebyshevSeries(const PhantomCiphertext& ct, const PhantomContext& cc,
                                                  const std::vector<double>& coeffs) const {
  std::vector<PhantomCiphertext> in(1);
  in[0] = ct;
  return std::move(chebyshev_lanes(std::move(in), cc, coeffs).at(0));
}

std::vector<PhantomCiphertext> FHECKKSRNS::chebyshev_lanes(std::vector<PhantomCiphertext> in, const PhantomContext& cc,
                                                           const std::vector<double>& coeffs) const {
  ChebEvaluator ev{cc, mul_key_, sf_, leaf_tables_};
  ev.B = in.size();
  for (auto& x : in)
    if (x.GetNoiseScaleDeg() > 1) EvalModReduceInPlace(cc, x, 1);
  ev.T.emplace(1, std::move(in));
  return ev.eval(coeffs);
}

void FHECKKSRNS::ApplyDoubleAngleIterations(PhantomCiphertext& ct, const PhantomContext& cc, uint32_t numIter) const {
  std::vector<PhantomCiphertext> v(1);
  v[0] = std::move(ct);
  double_angle_lanes(v, cc, numIter);
  ct = std::move(v[0]);
}

void FHECKKSRNS::double_angle_lanes(std::vector<PhantomCiphertext>& v, const PhantomContext& cc,
                                    uint32_t numIter) const {
  const int r = static_cast<int>(numIter);
  for (int j = 1; j <= r; ++j) {
    // 2 ct^2 - (2 pi)^(-2^(j - r)): doubling and constant folded in before the key switch; the
    // lanes' squarings share one batched key switch
    const double c = -1.0 / std::pow(2.0 * M_PI, std::pow(2.0, j - r));
    std::vector<MulAddJob> jobs;
    for (auto& ct : v) {
      if (ct.GetNoiseScaleDeg() > 1) EvalModReduceInPlace(cc, ct, 1);
      jobs.push_back(MulAddJob{&ct, &ct, 2, {}, c});
    }
    v = MulAddRescaleBatch(cc, jobs, mul_key_);
  }
}

std::vector<PhantomCiphertext> FHECKKSRNS::eval_mod_lanes(std::vector<PhantomCiphertext> in,
                                                          const PhantomContext& cc) const {
  std::vector<PhantomCiphertext> r = chebyshev_lanes(std::move(in), cc, cheb_);
  double_angle_lanes(r, cc, R_UNIFORM);
  return r;
}

PhantomCiphertext FHECKKSRNS::eval_mod(const PhantomCiphertext& ct, const PhantomContext& cc) const {
  std::vector<PhantomCiphertext> in(1);
  in[0] = ct;
  return std::move(eval_mod_lanes(std::move(in), cc).at(0));
}

PhantomCiphertext FHECKKSRNS::RaiseWithCorrection(const PhantomCiphertext& in, const PhantomContext& cc) const {
  PhantomCiphertext ct = in;
  if (ct.GetNoiseScaleDeg() > 1) EvalModReduceInPlace(cc, ct, 1);
  if (ct.coeff_modulus_size() < 2) throw std::invalid_argument("bootstrapping needs an input with at least two limbs");
  // scale the message down by 2^-correction and land on scale sf[0] (AdjustCiphertext)
  const double qdrop = static_cast<double>(cc.get_context_data(ct.chain_index()).moduli().back());
  const double s_raise = sf_.at(raise_level_);
  const double k = std::ldexp(1.0, -static_cast<int>(correction_)) * qdrop * s_raise / ct.scale();
  mult_by_real_integer_inplace(cc, ct, k);
  ct.SetNoiseScaleDeg(2);
  EvalModReduceInPlace(cc, ct, 1);
  ct.set_scale(s_raise);
  mod_switch_to_inplace(cc, ct, cc.size_Q());  // limb q0 only
  return RaiseMod(cc, ct, 1 + raise_level_);
}

// PHX_BOOT_TRACE=1: synchronise and report after every bootstrap stage (debugging aid)
static void trace(const PhantomContext& cc, const char* stage, const PhantomCiphertext& ct) {
  static const bool on = std::getenv("PHX_BOOT_TRACE") != nullptr;
  if (!on) return;
  static auto last = std::chrono::steady_clock::now();
  const hipError_t e = hipStreamSynchronize(cc.stream());
  const auto now = std::chrono::steady_clock::now();
  const double ms = std::chrono::duration<double, std::milli>(now - last).count();
  last = now;
  std::fprintf(stderr, "[boot] %-12s %8.3f ms  chain %zu limbs %zu scale %.6e deg %zu : %s\n", stage, ms,
               ct.chain_index(), ct.coeff_modulus_size(), ct.scale(), ct.GetNoiseScaleDeg(), hipGetErrorString(e));
}

std::vector<PhantomCiphertext> FHECKKSRNS::EvalBootstrapBatch(const std::vector<PhantomCiphertext>& in,
                                                              const PhantomContext& cc, int lanes,
                                                              uint32_t numSlots, size_t group) const {
  // a call from one of this function's own lane threads (a nested batch) runs serially on the
  // caller's lane: its lane streams are already in use by the outer batch
  static thread_local bool on_lane = false;
  const int k = on_lane ? 1 : std::max(1, std::min({lanes, PhantomContext::kLanes, static_cast<int>(in.size())}));
  if (group < 1 || group > static_cast<size_t>(phx::kLtGroupMax))
    throw std::invalid_argument("EvalBootstrapBatch: group must be 1.." + std::to_string(phx::kLtGroupMax));
  std::vector<PhantomCiphertext> out(in.size());
  // ciphertexts t, t + k, ... of lane t, up to `group` at a time in lockstep (shared plaintext
  // and key reads, EvalMod on 2 x group lanes).  A lane's m ciphertexts form ceil(m / group)
  // groups of near-equal size (43 at group 8: 8 + 5 x 7, not 5 x 8 + 3), so no lane ends on a
  // small group that shares its key and plaintext reads among few ciphertexts
  auto run_lane = [&](int t) {
    const Precom& pc = precom(numSlots, cc);
    std::vector<size_t> mine;
    for (size_t i = t; i < in.size(); i += k) mine.push_back(i);
    const size_t ng = (mine.size() + group - 1) / group;
    for (size_t gi = 0, g0 = 0; gi < ng; ++gi) {
      const size_t cnt = mine.size() / ng + (gi < mine.size() % ng ? 1 : 0);
      const size_t at = g0;
      g0 += cnt;
      if (cnt == 1) {
        out[mine[at]] = EvalBootstrap(in[mine[at]], cc, numSlots);
        continue;
      }
      std::vector<const PhantomCiphertext*> grp;
      for (size_t m = 0; m < cnt; ++m) grp.push_back(&in[mine[at + m]]);
      std::vector<PhantomCiphertext> r = bootstrap_group(grp, cc, pc);
      for (size_t m = 0; m < cnt; ++m) out[mine[at + m]] = std::move(r[m]);
    }
  };
  if (k == 1) {
    run_lane(0);
    return out;
  }
  const hipStream_t s0 = cc.stream();
  hipEvent_t fork;
  std::vector<hipEvent_t> join(k);
  PHX_CHECK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  for (auto& e : join) PHX_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  PHX_CHECK(hipEventRecord(fork, s0));
  for (int t = 0; t < k; ++t) PHX_CHECK(hipStreamWaitEvent(cc.lane_stream(t == 0 ? 0 : t), fork, 0));
  // lane t bootstraps ciphertexts t, t + k, ... from its own thread and streams; the inputs
  // (main-stream buffers) stay alive until the main stream has joined every lane
  std::vector<std::exception_ptr> err(k);
  std::vector<std::thread> workers;
  for (int t = 0; t < k; ++t)
    workers.emplace_back([&, t] {
      try {
        LaneGuard lane(cc, t);
        on_lane = true;
        run_lane(t);
      } catch (...) {
        err[t] = std::current_exception();
      }
    });
  for (auto& w : workers) w.join();
  hipError_t e = hipSuccess;
  for (int t = 0; t < k; ++t) {
    if (e == hipSuccess) e = hipEventRecord(join[t], cc.lane_stream(t));
    if (e == hipSuccess) e = hipStreamWaitEvent(s0, join[t], 0);
  }
  for (auto& c : out) c.retag(s0);
  bool failed = e != hipSuccess;
  for (auto& x : err) failed |= static_cast<bool>(x);
  if (failed) (void)hipDeviceSynchronize();
  (void)hipEventDestroy(fork);
  for (auto& j : join) (void)hipEventDestroy(j);
  for (auto& x : err)
    if (x) std::rethrow_exception(x);
  PHX_CHECK(e);
  return out;
}

PhantomCiphertext FHECKKSRNS::EvalBootstrap(const PhantomCiphertext& in, const PhantomContext& cc, uint32_t numSlots,
                                            uint32_t numIterations, uint32_t precision) const {
  const Precom& pc = precom(numSlots, cc);
  if (numIterations <= 1) return bootstrap_once(in, cc, pc);
  // iterative bootstrapping (bootstrap.cu:856-900): the first bootstrap's error, scaled up by
  // 2^precision, is bootstrapped again and subtracted
  if (precision < 1 || precision > 30) throw std::invalid_argument("iterative bootstrapping needs a precision in [1, 30]");
  const uint64_t pow2 = uint64_t(1) << precision;
  const size_t initSizeQ = in.coeff_modulus_size();
  PhantomCiphertext ctScaledUp = in;
  if (ctScaledUp.GetNoiseScaleDeg() > 1) EvalModReduceInPlace(cc, ctScaledUp, 1);
  MultByIntegerInPlace(cc, ctScaledUp, pow2);
  PhantomCiphertext ctInitialBootstrap = EvalBootstrap(in, cc, numSlots, numIterations - 1, precision);
  // (the reference rescales a pending product here; this engine's bootstraps return degree 1)
  if (ctInitialBootstrap.GetNoiseScaleDeg() > 1) EvalModReduceInPlace(cc, ctInitialBootstrap, 1);
  MultByIntegerInPlace(cc, ctInitialBootstrap, pow2);
  const size_t bootSizeQ = ctInitialBootstrap.coeff_modulus_size();
  if (bootSizeQ <= initSizeQ) return in;  // nothing gained: return the input, as the reference does
  // the bootstrapping error 2^p e at the input's level.  The reference drops limbs and subtracts
  // (ModSwitchLevelInPlace + EvalSubAuto), leaving the two operands at different FLEXIBLEAUTO
  // scales (sf[out] vs sf[in], 1.1e-4 apart at C4), which leaves 2^p m (sf_out/sf_in - 1) in the
  // error and caps the result near 13 bits; here EvalSubAuto brings the bootstrapped ciphertext
  // to the input's level and scale (integer mod-switch multiply + rescale) so 2^p m cancels.
  PhantomCiphertext ctBootstrappingError = ctInitialBootstrap;
  EvalSubAutoInplace(cc, ctBootstrappingError, ctScaledUp, sf_);
  PhantomCiphertext ctBootstrappedError = bootstrap_once(ctBootstrappingError, cc, pc);
  if (ctBootstrappedError.GetNoiseScaleDeg() > 1) EvalModReduceInPlace(cc, ctBootstrappedError, 1);
  PhantomCiphertext finalCiphertext = std::move(ctInitialBootstrap);
  EvalSubAutoInplace(cc, finalCiphertext, ctBootstrappedError, sf_);
  // scale back down by 2^precision
  EvalMultConstInplace(cc, finalCiphertext, 1.0 / static_cast<double>(pow2), sf_);
  EvalModReduceInPlace(cc, finalCiphertext, 1);
  return finalCiphertext;
}

std::vector<PhantomCiphertext> FHECKKSRNS::bootstrap_group(const std::vector<const PhantomCiphertext*>& in,
                                                           const PhantomContext& cc, const Precom& pc) const {
  const uint32_t N = static_cast<uint32_t>(cc.poly_degree()), M = 2 * N;
  const size_t K = in.size();
  if (pc.slots != N / 2 || K < 2) {
    std::vector<PhantomCiphertext> r;
    for (const PhantomCiphertext* c : in) r.push_back(bootstrap_once(*c, cc, pc));
    return r;
  }
  std::vector<PhantomCiphertext> x;
  for (const PhantomCiphertext* c : in) x.push_back(RaiseWithCorrection(*c, cc));
  auto level = [&](const LTLevel& lv) {
    std::vector<const PhantomCiphertext*> p;
    for (const PhantomCiphertext& c : x) p.push_back(&c);
    x = apply_level_group(cc, p, lv);
  };
  for (const LTLevel& lv : pc.enc) level(lv);
  // the conjugate split of each; EvalMod of all 2K halves in lockstep
  std::vector<PhantomCiphertext> halves(2 * K);
  for (size_t c = 0; c < K; ++c) {
    PhantomCiphertext& enc = x[c];
    PhantomCiphertext conj = EvalConjFused(cc, enc, galois_keys_);
    PhantomCiphertext enc_i = enc;
    sub_inplace(cc, enc_i, conj);
    add_inplace(cc, enc, conj);
    MultByMonomialInPlace(cc, enc_i, 3 * M / 4);  // times -i
    halves[2 * c] = std::move(enc);
    halves[2 * c + 1] = std::move(enc_i);
  }
  halves = eval_mod_lanes(std::move(halves), cc);
  for (size_t c = 0; c < K; ++c) {
    PhantomCiphertext im = std::move(halves[2 * c + 1]);
    MultByMonomialInPlace(cc, im, M / 4);  // times i
    x[c] = std::move(halves[2 * c]);
    EvalAddAutoInplace(cc, x[c], im, sf_);
  }
  for (const LTLevel& lv : pc.dec) level(lv);
  for (PhantomCiphertext& d : x) MultByIntegerInPlace(cc, d, uint64_t(1) << correction_);
  return x;
}

PhantomCiphertext FHECKKSRNS::bootstrap_once(const PhantomCiphertext& in, const PhantomContext& cc,
                                             const Precom& pc) const {
  const uint32_t N = static_cast<uint32_t>(cc.poly_degree()), M = 2 * N;
  const uint32_t slots = pc.slots;
  trace(cc, "start", in);
  PhantomCiphertext raised = RaiseWithCorrection(in, cc);
  trace(cc, "raise", raised);
  PhantomCiphertext dec;
  if (slots == N / 2) {
    // CoeffToSlot, then split the real and imaginary parts with one conjugation
    PhantomCiphertext enc = EvalCoeffsToSlots(raised, cc, slots);
    trace(cc, "cts", enc);
    PhantomCiphertext conj = EvalConjFused(cc, enc, galois_keys_);
    PhantomCiphertext enc_i = enc;
    sub_inplace(cc, enc_i, conj);
    add_inplace(cc, enc, conj);
    MultByMonomialInPlace(cc, enc_i, 3 * M / 4);  // times -i
    trace(cc, "conj-split", enc_i);
    // approximate modular reduction of both halves in lockstep: every product of the real and
    // the imaginary half shares one batched key switch (ChebEvaluator lanes, MulAddRescaleBatch)
    std::vector<PhantomCiphertext> halves(2);
    halves[0] = std::move(enc);
    halves[1] = std::move(enc_i);
    halves = eval_mod_lanes(std::move(halves), cc);
    enc = std::move(halves[0]);
    PhantomCiphertext im = std::move(halves[1]);
    MultByMonomialInPlace(cc, im, M / 4);  // times i
    trace(cc, "evalmod", enc);
    EvalAddAutoInplace(cc, enc, im, sf_);
    // SlotToCoeff
    dec = EvalSlotsToCoeffs(enc, cc, slots);
  } else {
    // sparse packing (bootstrap.cu:1044-1109).  PartialSum: the trace onto the subring of the
    // slots keeps the coefficients at multiples of N / (2 slots) (times that factor, which the
    // CoeffToSlot constants divide out)
    for (uint32_t j = 1; j * slots < N / 2; j <<= 1) {
      PhantomCiphertext t = EvalRotateFused(cc, raised, galois_keys_, static_cast<int>(j * slots));
      add_inplace(cc, raised, t);
    }
    trace(cc, "partial-sum", raised);
    // CoeffToSlot leaves w' = [c_lo | -i c_hi] (2 slots-periodic); w' + conj(w') = 2 [c_lo | c_hi]
    PhantomCiphertext enc = EvalCoeffsToSlots(raised, cc, slots);
    PhantomCiphertext conj = EvalConjFused(cc, enc, galois_keys_);
    add_inplace(cc, enc, conj);
    trace(cc, "cts", enc);
    enc = eval_mod(enc, cc);
    trace(cc, "evalmod", enc);
    // SlotToCoeff maps block 0 and block 1 to their halves of the embedding; the rotation by
    // `slots` adds them
    dec = EvalSlotsToCoeffs(enc, cc, slots);
    PhantomCiphertext r = EvalRotateFused(cc, dec, galois_keys_, static_cast<int>(slots));
    add_inplace(cc, dec, r);
  }
  trace(cc, "stc", dec);
  // undo the correction scaling
  MultByIntegerInPlace(cc, dec, uint64_t(1) << correction_);
  return dec;
}

}  // namespace phantom
