// dbow2_oracle.cc — CPU restatement of DBoW2's TemplatedVocabulary<FORB::TDescriptor, FORB>
// as ORB-SLAM2 uses it.  TEST INFRASTRUCTURE ONLY (see orb_oracle.h): the checker for the
// product's orbx_vocabulary_* functions, never linked into the product.
//
// Follows ORB_SLAM2/Thirdparty/DBoW2:
//   loadFromTextFile           TemplatedVocabulary.h:1338-1424
//   transform(features, v, fv, levelsup)   :1127-1198
//   transform(feature, word, weight, nid, levelsup)   :1218-1259
//   BowVector::addWeight / addIfNotExist / normalize   BowVector.cpp:38-98
//   FeatureVector::addFeature  FeatureVector.cpp:31-45
//   FORB::distance             FORB.cpp:81-101
//   ScoringObject::mustNormalize   ScoringObject.h:69-89
// Parity is pinned by the known-answer tests in tests/test_vocab_oracle.py (hand-computed
// trees) and by these sources; the reference's ORBvoc.txt is not in the tree, so no
// reference-produced vocabulary output exists to pin against.
//
// Two behaviours of the reference are undefined and are given a defined meaning here (and
// identically in the product):
//   * loadFromTextFile's `while(!f.eof())` runs once more after the final newline and appends
//     a phantom child of the root (pid, isLeaf and weight read as 0 under C++11, descriptor
//     left indeterminate by FORB::fromString).  The restatement stops at the last non-empty
//     line instead: an indeterminate descriptor cannot be reproduced.
//   * transform(feature, ...) leaves *nid unassigned when the descent reaches a leaf above
//     level L - levelsup; the caller's NodeId is then uninitialised.  Here nid = that leaf.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "orb_oracle.h"

namespace {

struct Node {
  int parent = 0;
  std::vector<int> children;
  uint8_t desc[32] = {0};
  double weight = 0;  // Node(): weight(0)
  uint32_t word_id = 0;  // Node(): word_id(0)
  bool is_leaf() const { return children.empty(); }
};

struct Voc {
  int k = 0, L = 0, scoring = 0, weighting = 0;
  std::vector<Node> nodes;
  std::vector<int> words;  // word id -> node id
};

int forb_distance(const uint8_t* a, const uint8_t* b) {
  int dist = 0;
  for (int i = 0; i < 8; i++) {
    uint32_t va, vb;
    memcpy(&va, a + 4 * i, 4);
    memcpy(&vb, b + 4 * i, 4);
    uint32_t v = va ^ vb;
    v = v - ((v >> 1) & 0x55555555);
    v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
    dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
  }
  return dist;
}

// ScoringObject.h:69-89 — (must normalize, L1?) per ScoringType
void must_normalize(int scoring, bool* must, bool* l1) {
  *must = scoring != 5;  // DOT_PRODUCT does not normalize
  *l1 = scoring != 1;    // L2_NORM uses L2, every other one L1
}

void transform_one(const Voc& V, const uint8_t* f, uint32_t* word, double* weight,
                   uint32_t* nid, int levelsup) {
  const int nid_level = V.L - levelsup;
  bool nid_set = false;
  if (nid_level <= 0) {
    *nid = 0;
    nid_set = true;
  }
  int final_id = 0, level = 0;
  do {
    ++level;
    const std::vector<int>& ch = V.nodes[final_id].children;
    final_id = ch[0];
    double best_d = forb_distance(f, V.nodes[final_id].desc);
    for (size_t c = 1; c < ch.size(); c++) {
      const double d = forb_distance(f, V.nodes[ch[c]].desc);
      if (d < best_d) {
        best_d = d;
        final_id = ch[c];
      }
    }
    if (level == nid_level) {
      *nid = (uint32_t)final_id;
      nid_set = true;
    }
  } while (!V.nodes[final_id].is_leaf());
  if (!nid_set) *nid = (uint32_t)final_id;  // see header: defined here, UB in the reference
  *word = V.nodes[final_id].word_id;
  *weight = V.nodes[final_id].weight;
}

}  // namespace

extern "C" {

void* oracle_voc_create(int k, int L, int scoring, int weighting, int n_nodes,
                        const int32_t* parent, const uint8_t* is_leaf, const uint8_t* desc,
                        const double* weight) {
  Voc* V = new Voc();
  V->k = k;
  V->L = L;
  V->scoring = scoring;
  V->weighting = weighting;
  V->nodes.resize(1);
  for (int i = 0; i < n_nodes; i++) {
    const int nid = (int)V->nodes.size();
    V->nodes.resize(nid + 1);
    Node& N = V->nodes[nid];
    N.parent = parent[i];
    if (parent[i] < 0 || parent[i] >= nid) {  // the reference indexes m_nodes[pid] unchecked
      delete V;
      return nullptr;
    }
    V->nodes[parent[i]].children.push_back(nid);
    memcpy(N.desc, desc + (size_t)i * 32, 32);
    N.weight = weight[i];
    if (is_leaf[i]) {
      N.word_id = (uint32_t)V->words.size();
      V->words.push_back(nid);
    }
  }
  return V;
}

// TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1338-1424)
void* oracle_voc_load_text(const char* path) {
  std::ifstream f(path);
  if (!f.is_open()) return nullptr;
  std::string s;
  std::getline(f, s);
  std::stringstream ss(s);
  int k = -1, L = -1, n1 = -1, n2 = -1;
  ss >> k >> L >> n1 >> n2;
  if (k < 0 || k > 20 || L < 1 || L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) return nullptr;
  std::vector<int32_t> parent;
  std::vector<uint8_t> leaf, desc;
  std::vector<double> weight;
  while (std::getline(f, s)) {
    if (s.find_first_not_of(" \t\r") == std::string::npos) continue;  // see header
    std::stringstream sn(s);
    int pid = 0, is_leaf = 0;
    sn >> pid >> is_leaf;
    uint8_t d[32] = {0};
    for (int i = 0; i < 32; i++) {
      int v;
      sn >> v;
      if (!sn.fail()) d[i] = (uint8_t)v;  // FORB::fromString keeps the byte on failure
    }
    double w = 0;
    sn >> w;
    parent.push_back(pid);
    leaf.push_back(is_leaf > 0);
    desc.insert(desc.end(), d, d + 32);
    weight.push_back(w);
  }
  return oracle_voc_create(k, L, n1, n2, (int)parent.size(), parent.data(), leaf.data(),
                           desc.data(), weight.data());
}

void oracle_voc_destroy(void* h) { delete (Voc*)h; }

void oracle_voc_info(const void* h, int* k, int* L, int* scoring, int* weighting, int* n_nodes,
                     int* n_words) {
  const Voc* V = (const Voc*)h;
  *k = V->k;
  *L = V->L;
  *scoring = V->scoring;
  *weighting = V->weighting;
  *n_nodes = (int)V->nodes.size();
  *n_words = (int)V->words.size();
}

// TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup)
// (TemplatedVocabulary.h:1127-1198).  word_of / node_of per feature (0xFFFFFFFF when the
// word's weight is <= 0, i.e. stopped); the BowVector and FeatureVector in key order.
void oracle_voc_transform(const void* h, const uint8_t* desc, int n, int levelsup,
                          uint32_t* word_of, uint32_t* node_of, uint32_t* bow_words,
                          double* bow_values, int* bow_n, uint32_t* fv_ids, int32_t* fv_off,
                          int32_t* fv_feats, int* fv_n) {
  const Voc& V = *(const Voc*)h;
  std::map<uint32_t, double> v;
  std::map<uint32_t, std::vector<uint32_t>> fv;
  for (int i = 0; i < n; i++) {
    if (word_of) word_of[i] = 0xFFFFFFFFu;
    if (node_of) node_of[i] = 0xFFFFFFFFu;
  }
  if (!V.words.empty()) {  // if(empty()) return;
    bool must, l1;
    must_normalize(V.scoring, &must, &l1);
    const bool tf = V.weighting == 0 || V.weighting == 1;  // TF_IDF or TF
    for (int i = 0; i < n; i++) {
      uint32_t id, nid;
      double w;
      transform_one(V, desc + (size_t)i * 32, &id, &w, &nid, levelsup);
      if (w > 0) {
        if (tf) {
          auto it = v.lower_bound(id);  // BowVector::addWeight
          if (it != v.end() && !(id < it->first)) it->second += w;
          else v.insert(it, {id, w});
        } else {
          auto it = v.lower_bound(id);  // BowVector::addIfNotExist
          if (it == v.end() || id < it->first) v.insert(it, {id, w});
        }
        fv[nid].push_back((uint32_t)i);  // FeatureVector::addFeature
        if (word_of) word_of[i] = id;
        if (node_of) node_of[i] = nid;
      }
    }
    if (tf && !v.empty() && !must) {
      const double nd = (double)v.size();
      for (auto& kv : v) kv.second /= nd;
    }
    if (must) {  // BowVector::normalize
      double norm = 0.0;
      if (l1) {
        for (auto& kv : v) norm += std::fabs(kv.second);
      } else {
        // the reference library is built -O3 -march=native (Thirdparty/DBoW2/CMakeLists.txt):
        // GCC contracts `norm += x * x` on FMA hosts
        for (auto& kv : v) norm = std::fma(kv.second, kv.second, norm);
        norm = std::sqrt(norm);
      }
      if (norm > 0.0)
        for (auto& kv : v) kv.second /= norm;
    }
  }
  int j = 0;
  for (auto& kv : v) {
    bow_words[j] = kv.first;
    bow_values[j] = kv.second;
    j++;
  }
  *bow_n = j;
  j = 0;
  int off = 0;
  fv_off[0] = 0;
  for (auto& kv : fv) {
    fv_ids[j] = kv.first;
    for (uint32_t f : kv.second) fv_feats[off++] = (int32_t)f;
    fv_off[++j] = off;
  }
  *fv_n = j;
}

}  // extern "C"
