// Shared by the kernels (common.h) and the host bindings.
#pragma once

// Batch assembly folded into a consumer kernel (the pipelined LSTM forward): rows perm[cursor * B + b] of up to
// 4 HBM-resident dataset tensors -> the static batch buffers, cursor advanced by the consumer's last workgroup
// (the same contract as mta_gather_batch, csrc/lstm_aux.hip).  src[0] is the window tensor x (windows, K, T, F).
struct MtaBatchGather {
  const float* src[4];
  float* dst[4];
  long row[4];  // floats per dataset row of each tensor
  int nt;       // tensors
  const int* perm;
  int* cursor;
  int B;        // windows per batch
};

