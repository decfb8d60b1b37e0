// Split topology as one batch instance: detection on one GPU, classification on another, crops handed
// over device to device (the arm-B analogue of the reference's detection -> classification gRPC hop,
// reference architectures/microservices/detection/app/grpc_client.py:126-168, which JPEG-encodes every
// crop and ships it through the host).
//
//   submit(imgs): detector executor (GPU i: letterbox -> YOLO -> decode -> NMS -> crop plan into
//                 BUF_XCROPS) ; classifier executor (GPU j) .submit_peer(): waits for the detector's
//                 slot on its own stream, pulls ctrl/meta/images, detections and the crop plan over
//                 xGMI (hipMemcpyPeerAsync), runs crop gather -> MobileNetV2 -> top-5
//   collect(s):   frees the detector slot, returns the classifier's complete result
//
// The dynamic batcher schedules it like any executor (csrc/runtime/batcher.cpp).
#pragma once
#include <map>
#include <memory>
#include <stdexcept>

#include "executor.h"
#include "peer.h"

namespace arena {

class SplitInstance : public BatchInstance {
 public:
  SplitInstance(std::shared_ptr<Executor> det, std::shared_ptr<Executor> cls) : det_(std::move(det)), cls_(std::move(cls)) {
    if (!det_ || !cls_) throw std::runtime_error("SplitInstance: null executor");
    if (!cls_->peer_stage()) throw std::runtime_error("SplitInstance: classifier executor is not a peer stage");
    // the classifier pulls the detector's slot over xGMI: refuse a pair without peer access at construction
    require_peer_access(cls_->device(), det_->device(), "SplitInstance", hip_can_access_peer);
  }
  std::vector<int> buckets() const override {
    std::vector<int> out;
    const auto c = cls_->buckets();
    for (int b : det_->buckets())
      for (int x : c)
        if (x == b) out.push_back(b);
    return out;
  }
  int num_slots() const override { return std::min(det_->num_slots(), cls_->num_slots()); }
  int max_det() const override { return cls_->max_det(); }
  int64_t raw_out_bytes() const override { return 0; }
  int64_t staging_bytes() const override { return det_->staging_bytes(); }
  int submit(const std::vector<InputImage>& imgs) override {
    const int a = det_->submit(imgs);
    int b;
    try {
      b = cls_->submit_peer(*det_, a);
    } catch (...) {
      det_->collect(a);
      throw;
    }
    det_slot_[b] = a;
    return b;
  }
  BatchResult collect(int slot) override {
    auto it = det_slot_.find(slot);
    if (it == det_slot_.end()) throw std::runtime_error("SplitInstance: unknown slot");
    const int a = it->second;
    det_slot_.erase(it);
    det_->collect(a);
    return cls_->collect(slot);
  }
  Executor& detector() { return *det_; }
  Executor& classifier() { return *cls_; }

 private:
  std::shared_ptr<Executor> det_, cls_;
  std::map<int, int> det_slot_;  // classifier slot -> detector slot (one instance thread uses this)
};

}  // namespace arena
