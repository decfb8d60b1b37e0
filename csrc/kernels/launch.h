// Host-side launch API for every HIP kernel of the arena (gfx950 only).
//
// Each launcher takes a plain parameter struct (device pointers + sizes) and a
// hipStream_t, and only enqueues work: no allocation, no synchronisation, so
// every launcher can be captured into a hipGraph by the executor
// (csrc/runtime/executor.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdexcept>
#include <string>

namespace arena {

// ---------------------------------------------------------------- conv (K2/K3/K4/K6/K10/K11/K13)
// Implicit-GEMM NHWC convolution on MFMA (v_mfma_f32_16x16x32_bf16) with a
// fused epilogue: + bias, activation, + residual, store into a channel slice
// of a concat buffer, optional second store nearest-upsampled x2 (FPN).
struct ImageMeta;
struct CropRef;
struct Ctrl;
struct ConvParams {
  const void* x;  // bf16 input, already offset to its channel slice
  int B, H, W;    // batch capacity and input spatial dims
  int xs;         // input pixel stride (elements)
  int Cin;        // input channels (multiple of 8)
  const void* w;  // bf16 weights [Cout_pad][Kpad], k = (kh*KW+kw)*Cin + ci
  int Kpad;       // multiple of 32
  const float* bias;  // fp32 [Cout_pad]
  void* y;            // output (bf16, or fp32 if f32out)
  int Ho, Wo, ys;     // output spatial dims and pixel stride (elements)
  int Cout;           // channels actually stored (multiple of 4)
  int Cout_pad;       // rows of w / bias (multiple of 16)
  int KH, KW, stride, pad_t, pad_l;
  const void* res;  // optional bf16 residual (same geometry as y), pixel stride rs
  int rs;
  void* y2;  // optional bf16 second output, 2x nearest upsampled, pixel stride y2s
  int y2s;
  int act;      // Act
  int f32out;   // store fp32 instead of bf16
  const int* bdev;  // optional live batch count on device
  int impl;         // kernel family for this call (0 = process default, see set_conv_impl)
  // Optional pointwise conv fused into the epilogue (3x3 halo-tile kernels only; YOLO Detect head):
  //   pw_y = W2 . act(conv(x) + bias) + pw_bias  (act2 = pw_act); the 3x3 result itself is not stored.
  // bf16: W2 [pw_cout_pad][pw_kpad], k = channel of the 3x3 output; fp32 (x3hg): pre-split planes with
  // permuted K columns (halo_x3g.hip), pw_y fp32.
  const void* pw_w;
  const float* pw_bias; // fp32 [pw_cout_pad]
  void* pw_y;           // bf16 output, pixel stride pw_ys
  int pw_ys, pw_cout, pw_kpad, pw_act;
  // Letterbox source (fp32 x3-h16 stem only): when lb_meta is set the input is not read from x but sampled
  // from the batch's uint8 images (letterbox.h), H x W being the space-to-depth grid (T / 2) of the target.
  const uint8_t* lb_pool;
  const ImageMeta* lb_meta;
  // fp32 programs: the weights pre-split into bf16 planes, [ceil(Kpad/32)][Cout_pad][h 32 | m 32 | l 32]
  // (engine/planner.py pack_conv_weight_x3), read by the x3g kernels (gemm_x3.hip); nullptr when absent
  const void* w3;
  // split-K x3g (kF32X3GSK): fp32 workspace for the partial tiles, splits x B x Ho x Wo x Cout_pad (executor: one
  // per slot and lane); sk_splits is set by the launcher
  float* sk_ws;
  int64_t sk_ws_bytes;
  int sk_splits;
};
void conv2d(const ConvParams& p, hipStream_t s);
void conv_igemm(const ConvParams& p, hipStream_t s);  // LDS-pipelined implicit GEMM (impl 3)
bool conv_pw(const ConvParams& p, hipStream_t s);     // 1x1 stride-1 fast path; false if unsupported
void set_conv_pw(bool v);                             // ARENA_CONV_PW=0 disables the fast path
bool conv3x3_v3(const ConvParams& p, hipStream_t s);  // 3x3 halo-tile v3; false if unsupported
bool conv_fc(const ConvParams& p, hipStream_t s);     // 1x1 conv on a 1x1 map, K 1280 (split-K FC); false if not
void set_conv_v3(bool v);                             // ARENA_CONV_V3=0 falls back to the v2 tile kernel
// Conv kernel family: 1 = direct global->VGPR loads, 2 = LDS-staged (default).
void set_conv_impl(int v);
int get_conv_impl();

// Exact-fp32 pipeline (csrc/kernels/conv_f32.hip): the same ConvParams geometry and epilogue with fp32
// activations, fp32 weights [Cout_pad][Kpad] (Kpad a multiple of 16) and v_mfma_f32_16x16x4_f32 (one
// rounding per product, fp32 accumulation: the reference's ONNX Runtime fp32 numerics).
// fp32 conv ConvParams.impl values beyond the families 0 (policy) / 1 (direct) / 2 (LDS): 10 + v selects LDS
// implicit-GEMM tile variant v < kF32Variants (conv_f32.hip launch_lds_variant), kF32Halo the 3x3 halo kernel.
// kF32X3 + v the fp32-accurate triple-bf16-split implicit GEMM variant v < kF32X3Variants (launch_x3_variant).
constexpr int kF32Variants = 16;
constexpr int kF32X3 = 40;
constexpr int kF32X3Variants = 12;
constexpr int kF32Halo = 100;
constexpr int kF32X3Halo = 101;  // 3x3 stride-1 halo tiles with the triple-bf16 split
constexpr int kF32X3HaloN3 = 102;  // ... with 48-channel tiles
constexpr int kF32X3HaloN2 = 103;  // ... with 32-channel tiles
constexpr int kF32Stream = 104;    // weight-stationary streaming conv, triple-bf16 split (Cin % 8, Kpad <= 192)
constexpr int kF32StreamN2 = 105;  // ... with 32-channel tiles
constexpr int kF32Fc = 106;        // split-K FC over a 1x1 map (fc_splitk.hip), exact fp32
constexpr int kF32StreamExact = 107;  // streaming small-K conv on exact fp32 MFMA (no split)
constexpr int kF32X3Halo16 = 108;    // x3 halo tiles of 16 x 16 output pixels (8 waves)
constexpr int kF32X3Halo16N3 = 109;  // ... with 48-channel tiles
constexpr int kF32X3H16 = 110;       // x3 3x3 stride-1 conv over exactly 16 input channels (s2d stems)
constexpr int kF32X3G = 111;         // x3g: 32x32x16 MFMA implicit GEMM over pre-split weights, variant v
constexpr int kF32X3GVariants = 20;  // v >= 10: v - 10 with the interleaved schedule   // impl kF32X3G + v, v < kF32X3GVariants (gemm_x3.hip XG_VARIANTS)
void x3_halo_prepare();
bool x3g_supported(const ConvParams& p);
bool conv_x3g(const ConvParams& p, hipStream_t s, int v);  // false if the conv or variant is not supported
// split-K x3g for small grids (bucket-1 latency): variant v = tile x splits (gemm_x3.hip XG_SK_VARIANTS); false when
// the workspace is missing or too small
constexpr int kF32X3GSK = 171;
constexpr int kF32X3GSKVariants = 9;
bool conv_x3g_sk(const ConvParams& p, hipStream_t s, int v);
void x3g_prepare();
// x3hg: 3x3 stride-1 halo tiles on 32x32x16 MFMAs over the same pre-split weights (halo_x3g.hip), variant v
constexpr int kF32X3HG = 131;
constexpr int kF32X3HGVariants = 14;
bool x3hg_supported(const ConvParams& p);
bool conv_x3hg(const ConvParams& p, hipStream_t s, int v);  // false if the conv or variant is not supported
void x3hg_prepare();
// ... with the Detect head's final 1x1 fused into the epilogue (ConvParams.pw_*, fp32), variant v
constexpr int kF32X3HGPw = 145;
constexpr int kF32X3HGPwVariants = 6;
// ... two more fused-1x1 tiles of 8 x 8 pixels on 2 waves (more workgroups for bucket 1 / 2): variants 6, 7
constexpr int kF32X3HGPwSmall = 181;
constexpr int kF32X3HGPwSmallVariants = 2;
bool conv_x3hg_pw(const ConvParams& p, hipStream_t s, int v);
// x3hr: the x3hg tiles with per-wave register weights (no weight LDS stage, two barriers per 16-channel chunk),
// variant v; and with the fused Detect-head 1x1
constexpr int kF32X3HR = 151;
constexpr int kF32X3HRVariants = 10;
constexpr int kF32X3HRPw = 161;
constexpr int kF32X3HRPwVariants = 6;
bool conv_x3hr(const ConvParams& p, hipStream_t s, int v);
bool conv_x3hr_pw(const ConvParams& p, hipStream_t s, int v);
bool conv_fc_f32(const ConvParams& p, hipStream_t s);
void conv2d_f32(const ConvParams& p, hipStream_t s);

// ---------------------------------------------------------------- depthwise 3x3 (K12)
struct DwParams {
  const void* x;
  int B, H, W, xs, C;
  const void* w;  // bf16 [9][C]
  const float* bias;
  void* y;
  int Ho, Wo, ys, stride, act;
  const int* bdev;
};
void dwconv3x3(const DwParams& p, hipStream_t s);
void dwconv3x3_f32(const DwParams& p, hipStream_t s);  // fp32 activations, fp32 weights [9][C]

// ---------------------------------------------------------------- fused inverted residual (K11+K12)
// MobileNetV2 block: 1x1 expand (+ReLU6) -> 3x3 depthwise stride S (+ReLU6)
// -> 1x1 project (+ residual).  The expanded and depthwise tensors live only
// in LDS (one output tile per workgroup, hidden channels in chunks of 32).
struct IrParams {
  const void* x;            // NHWC bf16 view (base already at its channel offset)
  int x_cs, H, W;
  int inp, inp_pad;         // inp_pad: multiple of 32
  int hid_pad;              // multiple of 32 (no-expand blocks: == inp_pad)
  int oup, oup_pad;         // oup_pad: multiple of 16
  int stride, expand, res;
  const void* we;           // bf16 [hid_pad][inp_pad]
  const float* be;          // [hid_pad]
  const void* wd;           // bf16 [9][hid_pad]
  const float* bd;          // [hid_pad]
  const void* wp;           // bf16 [oup_pad][hid_pad]
  const float* bp;          // [oup_pad]
  void* y;
  int y_cs, Ho, Wo;
  int B;
  const int* bdev;
  int x3w;                  // fp32: we / wp pre-split into bf16 [h|m|l] planes for ir_crop_f32.hip
  // Hidden-sliced 14x14 blocks (ir_crop_f32.hip only; 0 / 1 = a plain tensor): the input holds x_parts partial
  // sums at channel offsets j * inp (the block input is their sum, j = 0, 1, ... in order), and the block's
  // hidden channels are split over y_parts workgroups per band, each writing its partial output at channel
  // offset j * oup (partial 0 carries the project bias and the residual).
  int x_parts, y_parts;
  // fp32 classifier front end (stem = 1, t = 1 blocks, ir_f32.hip): X is not read from memory but built per
  // tile from the batch's uint8 images: crop gather + ImageNet normalisation (crop_gather_s2d semantics) into a
  // space-to-depth tile in LDS, then the 2x2 stem conv over it (+ bias, ReLU6; zero outside the H x W map).
  int stem;
  const uint8_t* st_pool;
  const ImageMeta* st_meta;
  const CropRef* st_crops;
  const Ctrl* st_ctrl;
  int st_S;                 // crop side (224): the stem map is st_S / 2 = H
  float st_mean[3], st_inv_std[3];
  const float* st_w;        // fp32 [inp_pad][64], k = (a * 2 + b) * 16 + c over the s2d input
  const float* st_b;        // fp32 [inp_pad]
};
void ir_block(const IrParams& p, hipStream_t s);
// Exact-fp32 fused block (csrc/kernels/ir_f32.hip): fp32 views / weights; we [hid_pad][inp_pad],
// wd [9][hid_pad], wp [oup_pad][hid_pad] fp32; inp_pad % 16, hid_pad % 32, oup_pad in {16, 32, 64, 96}.
void ir_block_f32(const IrParams& p, hipStream_t s);
bool ir_block_f32_supported(int stride, int inp_pad, int hid_pad, int oup_pad, int expand);
// Whole-map fp32-accurate block for the 14x14 / 7x7 stages (csrc/kernels/ir_crop_f32.hip, triple-bf16-split
// MFMA); ir_block_f32 dispatches blocks with split-plane weights (x3w, set by the planner) to it.
bool ir_block_crop_f32(const IrParams& p, hipStream_t s);
bool ir_block_crop_f32_supported(int H, int stride, int inp_pad, int hid_pad, int oup_pad, int expand);
// Tiled fp32-accurate x3 block for the >= 28x28 stages (csrc/kernels/ir_tile_x3.hip), also behind x3w
bool ir_tile_x3(const IrParams& p, hipStream_t s);
bool ir_tile_x3_supported(int stride, int inp_pad, int hid_pad, int oup_pad, int expand);
void ir_tile_x3_prepare();
bool ir_stem_x3(const IrParams& p, hipStream_t s);  // IrParams.stem with x3w: split-plane stem / project weights
void ir_prepare();
void set_ir_t14(bool v);  // ARENA_IR_T14=1: stride-1 14x14 blocks use one whole-crop tile
void set_ir_crop(bool v);
void set_ir_crop_split(int v);  // ARENA_IR_CROP_SPLIT: workgroups per crop in ir_crop (1 or 2)  // ARENA_IR_CROP=0: 7x7-output blocks use the tile kernel (ir_crop.hip)
void set_ir_wave(bool v);
void set_irx_slices_big(int n);  // hidden slices at most for crop capacities > 32 (< 1: ARENA_IRX_SLICES_BIG, default 2)
void set_irx_parts(int n);  // row bands per crop of the 14x14 whole-map fp32 IR kernel (2, 3, 4; else auto)  // ARENA_IR_WAVE=0: stride-1 blocks use the block-cooperative kernel

// ---------------------------------------------------------------- fused C3 block (K2/K3/K4 at 160x160 / 80x80)
// cv1|cv2 (1x1) -> NB x Bottleneck(1x1, 3x3 [+res]) -> cv3 (1x1) with every intermediate in LDS
// (csrc/kernels/c3_fused.hip).  Weight layouts as the conv kernels ([Cout_pad][Kpad], k = tap*C + c);
// the bottleneck 1x1 weights are [CH][32] (zero columns past CH).
struct C3Params {
  const void* x;  // bf16 NHWC input view, pixel stride xs
  int xs;
  int B, H, W;    // output size == input size (stride 1)
  const int* bdev;
  int C1, CH, NB, res;
  const void* w12;  // [2CH][C1]
  const float* b12;
  const void* wb1[2];  // [CH][32]
  const float* bb1[2];
  const void* wb2[2];  // [CH][round32(9*CH)]
  const float* bb2[2];
  const void* w3;   // [2CH][2CH]
  const float* b3;
  void* y;          // bf16 NHWC output view, pixel stride ys, 2CH channels
  int ys;
};
bool c3_fused_supported(int C1, int CH, int NB, bool res, int H, int W);
// fp32 form (csrc/kernels/c3_x3.hip): fp32 x / y, weights as pre-split bf16 planes [rows][3][K] (w12 [32][3][32],
// wb1 [16][3][16], wb2 [16][3][160] with k = tap * 16 + c, w3 [32][3][32]); the 160x160 block only.
bool c3_x3_supported(int C1, int CH, int NB, bool res, int H, int W);
void c3_x3(const C3Params& p, hipStream_t s);
void c3_x3_prepare();
void c3_fused(const C3Params& p, hipStream_t s);

// ---------------------------------------------------------------- SPPF pools (K5)
// x: [B,H,W] channels [0,C) of a buffer with pixel stride xs; writes the
// cascaded 5x5 max pools (== 5/9/13 windows) into channel slices C, 2C, 3C.
struct SppfParams {
  void* buf;
  int B, H, W, xs, C;
  const int* bdev;
};
void sppf_pool(const SppfParams& p, hipStream_t s);
void sppf_pool_f32(const SppfParams& p, hipStream_t s);  // fp32 buffer

// ---------------------------------------------------------------- image metadata
// Per-image record produced on the host for a batch (lives in device memory).
struct ImageMeta {
  int64_t offset;  // byte offset of the RGB uint8 HWC image in the image pool
  int h, w;        // original size
  int new_w, new_h;
  int pad_w, pad_h;
  float scale;     // letterbox scale
  float pad_[3];
};
static_assert(sizeof(ImageMeta) == 48, "ImageMeta layout");

// Control block shared by the pipeline kernels of one batch.
struct Ctrl {
  int n_images;    // live images (host-written)
  int n_crops;     // crops to classify in this pass (device-written)
  int crop_base;   // first crop of this pass (host-written for overflow passes)
  int total_crops; // all crops of the batch (device-written)
  int pad_[12];
};

// ---------------------------------------------------------------- letterbox (K1)
// Bilinear (cv2 INTER_LINEAR geometry) resize + pad(114) + /255 and
// space-to-depth(2): out [B, T/2, T/2, 16] bf16, channel (p*2+q)*3+c, 12..15 = 0.
struct LetterboxParams {
  const uint8_t* pool;
  const ImageMeta* meta;
  const Ctrl* ctrl;
  void* out;
  int B, T;
  int f32;  // fp32 output (exact-fp32 pipeline) instead of bf16
};
void letterbox_s2d(const LetterboxParams& p, hipStream_t s);

// fp32 NCHW [3,S,S] tensors in the image pool -> space-to-depth bf16.
struct TensorInParams {
  const uint8_t* pool;
  const ImageMeta* meta;
  const Ctrl* ctrl;
  void* out;
  int B, S;
  int f32;
};
void tensor_in_s2d(const TensorInParams& p, hipStream_t s);

// ---------------------------------------------------------------- detect decode (K7)
struct Candidate {
  float x1, y1, x2, y2;  // letterbox coordinates
  float score;
  int cls;
  int anchor;
  int pad_;
};
struct DecodeParams {
  // Per level l: head output [B, H_l, W_l] with 144 channels (64 DFL box + 80 cls), stride xs_l
  const void* head[3];
  int hw[3];      // H_l (== W_l)
  int xs[3];
  float stride[3];
  int B;
  float conf_thr;
  Candidate* cand;  // [B][cand_cap]
  int* cand_count;  // [B]
  int cand_cap;
  const Ctrl* ctrl;
  int f32;  // head activations are fp32
};
void detect_decode(const DecodeParams& p, hipStream_t s);

// Raw [84, A] fp32 detector output per image (reference ONNX contract).
struct YoloRawParams {
  const void* head[3];
  int hw[3];
  int xs[3];
  float stride[3];
  int B;
  void* out;          // image b at out + b * out_stride
  size_t out_stride;  // bytes
  const Ctrl* ctrl;
  int f32;
};
void yolo_raw(const YoloRawParams& p, hipStream_t s);

// ---------------------------------------------------------------- NMS (K8)
struct Detection {
  float x1, y1, x2, y2;  // original-image coordinates, clipped
  float conf;
  int cls;
  float pad_[2];
};
struct NmsParams {
  const Candidate* cand;
  const int* cand_count;
  int cand_cap;
  const ImageMeta* meta;
  int B;
  float iou_thr;
  Detection* det;  // [B][max_det]
  int* det_count;  // [B] (kept, possibly > max_det)
  int max_det;
  const Ctrl* ctrl;
};
void nms(const NmsParams& p, hipStream_t s);

// One-time kernel attribute setup (dynamic LDS > 64 KiB for NMS).  Must run
// before any hipGraph capture that contains the kernels.
void prepare_kernels();

// ---------------------------------------------------------------- crop plan + gather (K9)
struct CropRef {
  int img;
  int x1, y1, x2, y2;  // int-truncated, clamped; x2<=x1 or y2<=y1 => 1x1 black crop
  int det;             // index into the image's detections
  int pad_[2];
};
struct CropPlanParams {
  Detection* det;
  int* det_count;
  int max_det;
  const ImageMeta* meta;
  int B;
  CropRef* crops;  // [B*max_det]
  Ctrl* ctrl;
  int crop_cap;    // crops one classification pass can hold
  int whole;       // 1: every image is one crop (classifier-only programs); writes det/det_count
};
void crop_plan(const CropPlanParams& p, hipStream_t s);

struct CropGatherParams {
  const uint8_t* pool;
  const ImageMeta* meta;
  const CropRef* crops;
  const Ctrl* ctrl;
  void* out;  // [cap, S/2, S/2, 16] bf16 (space-to-depth, ImageNet-normalised)
  int cap, S;
  float mean[3], inv_std[3];
  int f32;
};
void crop_gather_s2d(const CropGatherParams& p, hipStream_t s);

// ---------------------------------------------------------------- fused preprocessing + stem conv
// src 0: letterbox (images) -> YOLOv5nu stem (3x3 over s2d, 16 -> 16, SiLU);
// src 1: crop gather (crops) -> MobileNetV2 stem (2x2 over s2d, 16 -> 32, ReLU6).
// The s2d input tile lives only in LDS (csrc/kernels/stem_fused.hip).
struct StemFusedParams {
  int src;                  // 0 letterbox, 1 crop gather
  const uint8_t* pool;
  const ImageMeta* meta;
  const Ctrl* ctrl;         // live counts (n_images / n_crops, crop_base)
  const CropRef* crops;     // src 1
  int cap;                  // batch capacity (images or crops)
  int S;                    // full-resolution side (letterbox T / crop S); output map is S/2 x S/2
  float mean[3], inv_std[3];  // src 1
  int KS;                   // stem kernel size over the s2d map (3 or 2)
  const void* w;            // bf16 [Cout][Kpad], k = tap*16 + c
  int Kpad;
  const float* bias;
  int Cout;
  void* y;                  // bf16 [cap, S/2, S/2, ys] (unused when w2 is set)
  int ys;
  int act;
  // Optional second conv (detector only): 3x3 stride 2, 16 -> Cout2, pad 1, on the stem output, which then
  // stays in LDS; y2 = bf16 [cap, S/4, S/4, y2s].
  const void* w2;           // bf16 [Cout2][Kpad2], k = tap*16 + c
  int Kpad2;
  const float* bias2;
  int Cout2, act2;
  void* y2;
  int y2s;
  // Optional first inverted residual (classifier only; t = 1: depthwise 3x3 + ReLU6 on the 32-channel stem
  // output, then project 32 -> 16, no residual) on the stem output kept in LDS; ir_y = bf16 [cap, S/2, S/2, ir_ys].
  // Layouts as ir_block: wd [9][32] bf16, bd [32] fp32, wp [16][32] bf16, bp [16] fp32.
  const void* ir_wd;
  const float* ir_bd;
  const void* ir_wp;
  const float* ir_bp;
  void* ir_y;
  int ir_ys;
};
void stem_fused(const StemFusedParams& p, hipStream_t s);
// fp32 detector front end (csrc/kernels/stem_x3.hip): letterbox -> stem -> 3x3 s2 conv with the stem map only in
// LDS; w = pre-split stem planes / 255 [3 ky][2 slabs][16][3][32], w2 = pre-split [9 taps][32][3][16], y2 fp32
void stem_s2_f32(const StemFusedParams& p, hipStream_t s);
void stem_s2_f32_prepare();

// ---------------------------------------------------------------- classification head (K13/K14)
struct AvgPoolParams {
  const void* x;
  int B, HW, C;
  void* y;  // [B][C], bf16 (or fp32 with f32)
  const int* bdev;
  int f32;
};
void global_avgpool(const AvgPoolParams& p, hipStream_t s);

// MobileNetV2 head 1x1 conv + activation fused with the global average pool (csrc/kernels/head_pool.hip):
// y[b][n] = mean_p act(sum_k x[b][p][k] w[n][k] + bias[n]), bf16 out.
struct HeadPoolParams {
  const void* x;            // bf16 [B][HW][xs]
  int xs, HW, K;            // K = input channels (<= Kpad)
  const void* w;            // bf16 [Npad][Kpad]
  int Kpad;
  const float* bias;        // [Npad]
  int N, Npad;
  void* y;                  // bf16 [B][ys]
  int ys;
  int act;
  int B;
  const int* bdev;
};
void head_pool(const HeadPoolParams& p, hipStream_t s);
// fp32 programs (x fp32 [B][HW][xs], w fp32 [Npad][Kpad], y fp32): triple-bf16-split MFMA, fp32-level error
void head_pool_f32(const HeadPoolParams& p, hipStream_t s);
void head_pool_f32_prepare();

struct TopkResult {
  int idx[5];
  float logit[5];
  float prob[5];
  int pad_;
};
struct TopkParams {
  const float* logits;  // [B][ld]
  int B, N, ld;
  TopkResult* out;       // written at out[ctrl->crop_base + i] when ctrl != null
  const Ctrl* ctrl;
  const int* bdev;
};
void topk_softmax(const TopkParams& p, hipStream_t s);

// Graph-safe memset replacement (kernel node).
void zero_fill(void* ptr, size_t bytes, hipStream_t s);
// One 64-bit device wall-clock stamp at `dst` (a kernel node: stage timing inside a captured graph).
void stamp(void* dst, hipStream_t s);

// Device half of the split JPEG decoder (csrc/kernels/jpeg_idct.hip): for n_images descriptors (jpeg_desc.h)
// reconstruct packed RGB at d_pool + desc.rgb_off from the quantized coefficient blocks at d_pool +
// comp.coef_off (sample planes at d_pool + comp.plane_off as scratch).  max_blocks / max_pixels: the largest
// total_blocks / width * height over the batch (grid sizes).
struct JpegDesc;
void jpeg_reconstruct(const JpegDesc* d_descs, uint8_t* d_pool, int n_images, int max_blocks, int64_t max_pixels,
                      hipStream_t s);

}  // namespace arena
