// orbx_vocab.h — device view of a DBoW2 vocabulary (orbx_vocab.hip) for the frame pipeline.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/orbx.h"

namespace orbx {

// Children of a node are contiguous records [child_begin, child_begin + nchild): descriptor
// (32 B) and meta {node id, that node's child_begin, its nchild, its word id}.
struct VocView {
  const uint8_t* cdesc;  // [n_nodes - 1][32]
  const int4* cmeta;     // [n_nodes - 1]
  const double* weight;  // [n_nodes] node weight (Node::weight)
  const double* word_weight;  // [n_words] weight of word w's node (m_words[w]->weight)
  int root_cb, root_nc;
  int n_words;
  int k;
};

// FeatureVector node table of one levelsup: possible FeatureVector nodes, ascending id
struct VocRanks {
  int levelsup = -1;
  int nb = 0;
  uint32_t* d_rank_of_node = nullptr;  // [n_nodes] rank, 0xFFFFFFFF if never a FeatureVector key
  uint32_t* d_rank_ids = nullptr;      // [nb] node id of rank b
};

// Pinned-host mirrors of a one-image call's outputs (the resident drop-in transform): the
// kernels write them beside their device outputs, so no download copy runs.  All nullable.
struct VocHostOut {
  uint8_t* desc_copy;                     // k_voc_transform: the descriptors it read (device)
  uint32_t* word_of;                      // k_voc_transform: word id, FeatureVector node id
  uint32_t* node_of;
  uint32_t* words;                        // k_bowfv: BowVector
  double* values;
  int* nwords;
  uint32_t* ids;                          // k_bowfv: FeatureVector CSR
  int* off;
  int* feats;
  int* nn;
};

int vocab_view(const orbx_vocabulary* voc, VocView* v, int* device);
int vocab_ranks(const orbx_vocabulary* voc, int levelsup, const VocRanks** out);

// Per feature of every image: word id, FeatureVector rank and node id (0xFFFFFFFF when
// stopped; d_node_of nullable), and the weight of the node the descent ended on.
int launch_voc_transform(const VocView& V, int nid_level, const uint32_t* d_rank_of_node,
                         const uint8_t* d_desc, int64_t desc_stride_img, const int* d_counts,
                         int n_fixed, int max_n, uint32_t* d_word_of, uint32_t* d_rank_of,
                         uint32_t* d_node_of, double* d_weight_of, int64_t out_stride_img,
                         int nimg, hipStream_t s, const VocHostOut& ho = VocHostOut{});
// BowVector of every image from the word ids and weights (TemplatedVocabulary.h:1144-1197).
// max_n <= 8192.
int launch_bowvec(int scoring, int weighting, const uint32_t* d_word_of,
                  const double* d_weight_of, int64_t in_stride, const int* d_counts, int n_fixed,
                  int max_n, uint32_t* d_words, double* d_values, int64_t out_stride,
                  int* d_nwords, int nimg, hipStream_t s);
// BowVector (as launch_bowvec) and FeatureVector CSR (as launch_csr with id_lo 0 over
// d_rank_ids) of every image in one launch (k_bowfv).  ORBX_EUNSUPPORTED when it does not apply
// (more than 4096 features, or more than 2048 in a call of more than 4 images; ids too wide; no
// rank table): the caller then runs
// launch_bowvec + launch_csr.
int launch_bowfv(int scoring, int weighting, int n_words, const uint32_t* d_word_of,
                 const uint32_t* d_rank_of, const double* d_weight_of, int64_t in_stride,
                 const int* d_counts, int n_fixed, int max_n, uint32_t* d_words, double* d_values,
                 int64_t out_stride, int* d_nwords, int nb, const uint32_t* d_rank_ids,
                 uint32_t* d_ids, int* d_off, int* d_feats, int64_t feats_stride, int* d_nn,
                 int nimg, hipStream_t s, const VocHostOut& ho = VocHostOut{});

}  // namespace orbx
