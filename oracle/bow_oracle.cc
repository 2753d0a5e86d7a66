// ORACLE (test infrastructure only): CPU restatement of the DBoW2 pieces
// Frame::ComputeBoW runs (frame.cc:761-766): the ORB vocabulary's text loader
// and transform(features, BowVector&, FeatureVector&, levelsup).  Only tests/
// and bench.py's side lines use it, as the checker.
//
// Restated from 3rdparty/DBoW2/DBoW2 (file:line):
//   * TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1248-1327):
//     header "k L scoring weighting" (rejected outside k<=20, 1<=L<=10,
//     scoring<=5, weighting<=3); then, until eof, one node per getline: parent,
//     isLeaf flag, 32 descriptor tokens (FORB::fromString, FORB.cpp:105-116:
//     ints stored as uchar, a failed read leaves the byte), weight.  Node ids
//     are line order; children are pushed in line order; a node is a word iff
//     its flag is > 0 (word ids in line order) but isLeaf() means "no
//     children" (:334).  A final empty line (file ending in '\n') still makes
//     a node: C++11 extraction failures store 0, so it is a childless
//     non-word child of the root with weight 0; its descriptor bytes are
//     uninitialised in the reference (cv::Mat::create), zero here.
//   * transform per feature (:1140-1179): descend from the root taking the
//     first strict minimum of FORB::distance (FORB.cpp:71-88) over the
//     children in order, until a node without children; record the node at
//     depth L - levelsup (root when <= 0; left unset by the reference when the
//     path is shorter -- UB there, 0 here).
//   * transform(features, v, fv, levelsup) (:1057-1118): TF / TF_IDF sum the
//     weights of a word in feature order (BowVector::addWeight,
//     BowVector.cpp:30-38), IDF / BINARY keep the first (addIfNotExist,
//     :42-48); zero-weight (stopped) words are skipped for both vectors;
//     FeatureVector::addFeature appends indices (FeatureVector.cpp:28-38).
//     Scoring L1 / CHI_SQUARE / KL / BHATTACHARYYA normalise L1, L2_NORM
//     normalises L2 (ScoringObject.h:76-91, BowVector::normalize :52-66: the
//     norm summed in word-id order); DOT_PRODUCT does not normalise, and then
//     TF / TF_IDF divide by the number of words.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

namespace {

struct Node {
  uint32_t parent = 0;
  double weight = 0;
  uint32_t word_id = 0;
  uint8_t desc[32] = {};
  std::vector<uint32_t> children;
};

struct Vocab {
  int k = 0, L = 0, scoring = 0, weighting = 0;
  std::vector<Node> nodes;
  uint32_t n_words = 0;
};

int desc_dist(const uint8_t* a, const uint8_t* b) {  // FORB::distance
  int d = 0;
  for (int i = 0; i < 8; ++i) {
    uint32_t pa, pb;
    std::memcpy(&pa, a + 4 * i, 4);
    std::memcpy(&pb, b + 4 * i, 4);
    uint32_t v = pa ^ pb;
    v = v - ((v >> 1) & 0x55555555u);
    v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
    d += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
  }
  return d;
}

bool load_text(const char* path, Vocab& V) {
  std::ifstream f(path);
  if (!f.is_open() || f.eof()) return false;
  std::string s;
  std::getline(f, s);
  std::stringstream hs(s);
  int n1 = 0, n2 = 0;
  hs >> V.k >> V.L >> n1 >> n2;
  if (V.k < 0 || V.k > 20 || V.L < 1 || V.L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3)
    return false;
  V.scoring = n1, V.weighting = n2;
  V.nodes.assign(1, Node());
  while (!f.eof()) {
    std::string line;
    std::getline(f, line);
    std::stringstream ls(line);
    const uint32_t nid = (uint32_t)V.nodes.size();
    V.nodes.emplace_back();
    int pid = 0;
    ls >> pid;
    if (pid < 0 || (uint32_t)pid >= nid) return false;  // out-of-range parent: UB in the reference
    V.nodes[nid].parent = (uint32_t)pid;
    V.nodes[pid].children.push_back(nid);
    int is_leaf = 0;
    ls >> is_leaf;
    std::stringstream ds;
    for (int i = 0; i < 32; ++i) {
      std::string tok;
      ls >> tok;
      ds << tok << " ";
    }
    std::stringstream dp(ds.str());
    for (int i = 0; i < 32; ++i) {
      int v;
      dp >> v;
      if (!dp.fail()) V.nodes[nid].desc[i] = (uint8_t)v;
    }
    double w = 0;
    ls >> w;
    V.nodes[nid].weight = w;
    if (is_leaf > 0) V.nodes[nid].word_id = V.n_words++;
  }
  return true;
}

void transform_one(const Vocab& V, const uint8_t* feat, int levelsup, uint32_t& word,
                   double& weight, uint32_t& nid) {
  const int nid_level = V.L - levelsup;
  nid = 0;
  uint32_t id = 0;
  int level = 0;
  do {
    ++level;
    const std::vector<uint32_t>& ch = V.nodes[id].children;
    id = ch[0];
    int best = desc_dist(feat, V.nodes[id].desc);
    for (size_t j = 1; j < ch.size(); ++j) {
      const int d = desc_dist(feat, V.nodes[ch[j]].desc);
      if (d < best) best = d, id = ch[j];
    }
    if (level == nid_level) nid = id;
  } while (!V.nodes[id].children.empty());
  word = V.nodes[id].word_id;
  weight = V.nodes[id].weight;
}

}  // namespace

extern "C" {

void* orc_vocab_load(const char* path) {
  auto* V = new Vocab();
  if (!load_text(path, *V)) {
    delete V;
    return nullptr;
  }
  return V;
}

void orc_vocab_free(void* v) { delete static_cast<Vocab*>(v); }

void orc_vocab_info(const void* v, int* info) {
  const Vocab& V = *static_cast<const Vocab*>(v);
  info[0] = V.k, info[1] = V.L, info[2] = V.scoring, info[3] = V.weighting;
  info[4] = (int)V.nodes.size(), info[5] = (int)V.n_words;
}

// transform(features, BowVector&, FeatureVector&, levelsup)
void orc_bow_transform(const void* v, const uint8_t* descs, int n, int levelsup,
                       uint32_t* bow_words, double* bow_weights, int* n_words, uint32_t* fv_nodes,
                       int32_t* fv_offsets, uint32_t* fv_features, int* n_nodes) {
  const Vocab& V = *static_cast<const Vocab*>(v);
  std::map<uint32_t, double> bow;
  std::map<uint32_t, std::vector<uint32_t>> fv;
  if (V.n_words > 0) {
    const bool tf = V.weighting == 0 || V.weighting == 1;
    for (int i = 0; i < n; ++i) {
      uint32_t w, nid;
      double wt;
      transform_one(V, descs + 32 * (size_t)i, levelsup, w, wt, nid);
      if (!(wt > 0)) continue;
      auto it = bow.find(w);
      if (it == bow.end()) bow.emplace(w, wt);
      else if (tf) it->second += wt;
      fv[nid].push_back((uint32_t)i);
    }
    const bool must = V.scoring != 5;
    if (tf && !bow.empty() && !must) {
      const double nd = (double)bow.size();
      for (auto& e : bow) e.second /= nd;
    }
    if (must) {
      double norm = 0.0;
      if (V.scoring == 1) {
        for (auto& e : bow) norm = std::fma(e.second, e.second, norm);  // contracted in the reference
        norm = std::sqrt(norm);
      } else {
        for (auto& e : bow) norm += std::fabs(e.second);
      }
      if (norm > 0.0)
        for (auto& e : bow) e.second /= norm;
    }
  }
  int k = 0;
  for (auto& e : bow) bow_words[k] = e.first, bow_weights[k] = e.second, ++k;
  *n_words = k;
  int j = 0, off = 0;
  for (auto& e : fv) {
    fv_nodes[j] = e.first;
    fv_offsets[j] = off;
    for (uint32_t i : e.second) fv_features[off++] = i;
    ++j;
  }
  fv_offsets[j] = off;
  *n_nodes = j;
}

}  // extern "C"
