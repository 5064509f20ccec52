unit nnHip;
{ nnHip — the Pascal side of libtensorium_hip.so (MI355X / gfx950): every
  entry point of include/tns.h declared cdecl-external, a TNNHip<T> class
  with TNNCuda<T>'s method list (source/nncuda.pas:101-157) over the device
  backend (boundary B), initHIP mirroring initCUDART (ntensors.pas:6191-6210),
  and useHipOpTable binding the op-table drop-ins (boundary A) into the
  TTensor<Single> class-var pointers (ntensors.pas:345-385) the way
  TTensorOps.initSingle binds the USE_OPENBLAS / USE_MKL overrides
  (ntensors.pas:12735-12756).

  The library computes fp32 only: TNNHip<T> refuses any T but single.
  Entry points return a status (0 = TNS_OK); every call is checked and a
  failure raises ETnsError with tns_last_error(), as SAFE_CALL raises for
  CUDA (nncuda.pas:216-275).  Methods of TNNCuda<T> that are not on the
  SGEMM + im2col-convolution hot path (SURVEY.md §8: max-pool, dropout,
  SWISH, L2 / logistic cost, power, the NVRTC / CUBIN loaders) raise
  ENotSupportedException instead of silently doing nothing.

  tests/test_pascal_unit.py cross-checks every external declaration here
  against include/tns.h (name, parameter count, parameter widths, result). }

{$ifdef FPC}
{$mode Delphi}
{$PackRecords C}
{$endif}
{$PointerMath ON}
{$Z4}

interface

uses
  SysUtils;

const
  libtns = 'tensorium_hip';

  TNS_OK = 0;
  TNS_ERR_ARG = 1;
  TNS_ERR_HIP = 2;
  TNS_ERR_NOMEM = 3;
  TNS_ERR_UNSUPPORTED = 4;

  TNS_CONV_UNFUSED = 0;
  TNS_CONV_FUSED = 1;
  TNS_CONV_IM2COL = 2;
  TNS_CONV_IMPLICIT = 3;

  TNS_OP_GEMM = 0;
  TNS_OP_IM2COL = 1;
  TNS_OP_COL2IM = 2;
  TNS_OP_BIAS = 3;
  TNS_OP_ACTIVATE = 4;

  TNS_OPT_STRICT_BETA0 = 0;
  TNS_OPT_CONV_VARIANT = 1;
  TNS_OPT_CONV_PAD = 2;
  TNS_OPT_NT_SDOT = 3;
  TNS_OPT_SRSS_QUIRK = 4;
  TNS_OPT_TT_EXACT = 5;
  TNS_OPT_SDOT_FORM = 6;
  TNS_OPT_DX_FUSED = 7;
  TNS_OPT_DX_TILE = 8;
  TNS_OPT_DW_TILE = 9;
  TNS_OPT_BWD_OVERLAP = 10;
  TNS_OPT_DX_CONV = 11;
  TNS_OPT_DW_RES = 12;
  TNS_OPT_DERIVE_SUMS = 13;
  TNS_OPT_SCRATCH_CAP = 14;

type
  PTnsCtx = pointer;
  PPTnsCtx = ^PTnsCtx;
  THipMem = PSingle;                  { device pointer; offsets in ELEMENTS (TCUMem + offset) }
  PHipMem = ^THipMem;
  TTnsErrorHook = procedure(code: longint; msg: PAnsiChar); cdecl;
  ETnsError = class(Exception);

{ ---- library / error channel ------------------------------------------- }
function tns_abi_version(): longint; cdecl; external libtns;
function tns_last_error(): PAnsiChar; cdecl; external libtns;
procedure tns_clear_error(); cdecl; external libtns;
procedure tns_set_error_hook(hook: TTnsErrorHook); cdecl; external libtns;
function tns_device_count(): longint; cdecl; external libtns;

{ ---- A. op-table drop-ins (host pointers; ntensors.pas:345-385) ---------- }
procedure tns_cblas_sgemm(Order, TransA, TransB: longint; M, N, K: int64; ALPHA: single;
  A: PSingle; lda: int64; B: PSingle; ldb: int64; BETA: single; C: PSingle; ldc: int64);
  cdecl; external libtns;
procedure tns_cblas_sgemm_batch_strided(Layout, TransA, TransB: longint; M, N, K: int64;
  alpha: single; A: PSingle; lda, strideA: int64; B: PSingle; ldb, strideB: int64;
  beta: single; C: PSingle; ldc, strideC, batch_size: int64); cdecl; external libtns;
procedure tns_im2col(aChannels, aHeight, aWidth, kernelHeight, kernelWidth, padHeight,
  padWidth, strideY, strideX, dilationY, dilationX: int64; inData: PSingle; inOffset: int64;
  outData: PSingle; outOffset: int64; multiThread: boolean); cdecl; external libtns;
procedure tns_col2im(aChannels, aHeight, aWidth, kernelHeight, kernelWidth, padHeight,
  padWidth, strideY, strideX, dilationY, dilationX: int64; inData: PSingle; inOffset: int64;
  outData: PSingle; outOffset, batch: int64; multiThread: boolean); cdecl; external libtns;
procedure tns_im2col_strided_batched(aChannels, aHeight, aWidth, kernelHeight, kernelWidth,
  padHeight, padWidth, strideY, strideX, dilationY, dilationX: int64; im: PSingle;
  imStride, imOffset: int64; col: PSingle; colStride, colOffset, batchCount: int64);
  cdecl; external libtns;
procedure tns_col2im_strided_batched(aChannels, aHeight, aWidth, kernelHeight, kernelWidth,
  padHeight, padWidth, strideY, strideX, dilationY, dilationX: int64; inData: PSingle;
  inStride, inOffset: int64; outData: PSingle; outStride, outOffset, batchCount: int64);
  cdecl; external libtns;

{ ---- B. device backend (TNNCuda<T> twin; nncuda.pas:35-157) -------------- }
function tns_hip_create(deviceIndex: longint; ctx: PPTnsCtx): longint; cdecl; external libtns;
function tns_hip_destroy(ctx: PTnsCtx): longint; cdecl; external libtns;
function tns_hip_set_stream(ctx: PTnsCtx; hipStream: pointer): longint; cdecl; external libtns;
function tns_hip_get_stream(ctx: PTnsCtx): pointer; cdecl; external libtns;
function tns_hip_pending_dw(ctx: PTnsCtx): longint; cdecl; external libtns;
function tns_hip_finish(ctx: PTnsCtx): longint; cdecl; external libtns;
function tns_hip_malloc(ctx: PTnsCtx; nElements: int64; res: PHipMem): longint; cdecl; external libtns;
function tns_hip_free(ctx: PTnsCtx; p: THipMem): longint; cdecl; external libtns;
function tns_hip_write_buffer(ctx: PTnsCtx; dev: THipMem; bytes: int64; host: pointer): longint;
  cdecl; external libtns;
function tns_hip_read_buffer(ctx: PTnsCtx; dev: THipMem; bytes: int64; host: pointer): longint;
  cdecl; external libtns;
function tns_hip_gemm(ctx: PTnsCtx; transA, transB: boolean; M, N, K: int64; ALPHA: single;
  A: THipMem; aOffset, lda: int64; B: THipMem; bOffset, ldb: int64; BETA: single; C: THipMem;
  cOffset, ldc: int64): longint; cdecl; external libtns;
function tns_hip_gemm_batched(ctx: PTnsCtx; transA, transB: boolean; M, N, K: int64;
  ALPHA: single; A: PHipMem; aOffset, lda: int64; B: PHipMem; bOffset, ldb: int64;
  BETA: single; C: PHipMem; cOffset, ldc, batchCount: int64): longint; cdecl; external libtns;
function tns_hip_gemm_strided_batched(ctx: PTnsCtx; transA, transB: boolean; M, N, K: int64;
  ALPHA: single; A: THipMem; aOffset, lda, strideA: int64; B: THipMem; bOffset, ldb,
  strideB: int64; BETA: single; C: THipMem; cOffset, ldc, strideC, batchCount: int64): longint;
  cdecl; external libtns;
function tns_hip_im2col(ctx: PTnsCtx; aChannels, aHeight, aWidth, kernelHeight, kernelWidth,
  padHeight, padWidth, strideY, strideX, dilationY, dilationX: int64; im: THipMem;
  imOffset: int64; col: THipMem; colOffset: int64): longint; cdecl; external libtns;
function tns_hip_im2col_strided_batched(ctx: PTnsCtx; aChannels, aHeight, aWidth, kernelHeight,
  kernelWidth, padHeight, padWidth, strideY, strideX, dilationY, dilationX: int64; im: THipMem;
  imStride, imOffset: int64; col: THipMem; colStride, colOffset, batchCount: int64): longint;
  cdecl; external libtns;
function tns_hip_col2im(ctx: PTnsCtx; aChannels, aHeight, aWidth, kernelHeight, kernelWidth,
  padHeight, padWidth, strideY, strideX, dilationY, dilationX: int64; col: THipMem;
  colOffset: int64; im: THipMem; imOffset: int64): longint; cdecl; external libtns;
function tns_hip_col2im_strided_batched(ctx: PTnsCtx; aChannels, aHeight, aWidth, kernelHeight,
  kernelWidth, padHeight, padWidth, strideY, strideX, dilationY, dilationX: int64; col: THipMem;
  colStride, colOffset: int64; im: THipMem; imStride, imOffset, batchCount: int64): longint;
  cdecl; external libtns;
function tns_hip_forward_bias(ctx: PTnsCtx; dstSize: int64; dst: THipMem; offset, srcSize: int64;
  src: THipMem; incb, batch: int64): longint; cdecl; external libtns;
function tns_hip_backward_bias(ctx: PTnsCtx; dstSize: int64; dst: THipMem; srcSize: int64;
  src: THipMem; srcOffset, incb, batch: int64): longint; cdecl; external libtns;
function tns_hip_activate_array(ctx: PTnsCtx; N: int64; x: THipMem; offset: int64;
  activation: longint): longint; cdecl; external libtns;
function tns_hip_derive_array(ctx: PTnsCtx; N: int64; x: THipMem; offset: int64;
  activation: longint; delta: THipMem): longint; cdecl; external libtns;
function tns_hip_axpy(ctx: PTnsCtx; N: int64; a: single; x: THipMem; xOffset, incx: int64;
  y: THipMem; yOffset, incy: int64): longint; cdecl; external libtns;
function tns_hip_scale(ctx: PTnsCtx; N: int64; a: single; x: THipMem; stride: int64): longint;
  cdecl; external libtns;
function tns_hip_sgd_update(ctx: PTnsCtx; nWeights: int64; weights, weight_updates: THipMem;
  n: int64; biases, bias_updates, scales, scale_updates: THipMem; lrOverBatch,
  negDecayTimesBatch, momentum: single): longint; cdecl; external libtns;
function tns_hip_fill(ctx: PTnsCtx; N: int64; x: THipMem; offset: int64; val: single;
  stride: int64): longint; cdecl; external libtns;
function tns_hip_copy(ctx: PTnsCtx; N: int64; src: THipMem; srcOffset, inca: int64; dst: THipMem;
  dstOffset, incb: int64): longint; cdecl; external libtns;
function tns_hip_clamp(ctx: PTnsCtx; N: int64; alpha: single; src, dst: THipMem;
  stride, offset: int64): longint; cdecl; external libtns;
function tns_hip_addvv(ctx: PTnsCtx; N: int64; src1: THipMem; src1Offset, inca: int64;
  src2: THipMem; src2Offset, incb: int64; dst: THipMem; dstOffset, incc: int64): longint;
  cdecl; external libtns;
function tns_hip_subvv(ctx: PTnsCtx; N: int64; src1: THipMem; src1Offset, inca: int64;
  src2: THipMem; src2Offset, incb: int64; dst: THipMem; dstOffset, incc: int64): longint;
  cdecl; external libtns;
function tns_hip_mulvv(ctx: PTnsCtx; N: int64; src1: THipMem; src1Offset, inca: int64;
  src2: THipMem; src2Offset, incb: int64; dst: THipMem; dstOffset, incc: int64): longint;
  cdecl; external libtns;
function tns_hip_fmavv(ctx: PTnsCtx; N: int64; src1: THipMem; src1Offset, inca: int64;
  src2: THipMem; src2Offset, incb: int64; src3: THipMem; src3Offset, incc: int64; dst: THipMem;
  dstOffset, incd: int64): longint; cdecl; external libtns;
function tns_hip_fmavss(ctx: PTnsCtx; N: int64; src: THipMem; offset: int64; scalar,
  bias: single; dst: THipMem): longint; cdecl; external libtns;
function tns_hip_inverse_sqrt(ctx: PTnsCtx; N: int64; alpha: single; src, dst: THipMem;
  stride, offset: int64): longint; cdecl; external libtns;

{ non-convolutional YOLOv3 layers }
function tns_hip_shortcut(ctx: PTnsCtx; N: int64; a: THipMem; aOffset: int64; b: THipMem;
  bOffset: int64; output: THipMem; outOffset: int64; activation: longint): longint;
  cdecl; external libtns;
function tns_hip_upsample(ctx: PTnsCtx; aBatch, aChannels, outHeight, outWidth: int64;
  input: THipMem; stride: int64; isForward: longint; scale: single; output: THipMem;
  zeroIn: longint): longint; cdecl; external libtns;
function tns_hip_yolo_forward(ctx: PTnsCtx; batch, anchors, classes, hw: int64; input,
  output: THipMem): longint; cdecl; external libtns;

{ batch norm / softmax }
function tns_hip_means_and_vars(ctx: PTnsCtx; srcSize, dstSize, groups: int64; src: THipMem;
  offset: int64; means, vars: THipMem): longint; cdecl; external libtns;
function tns_hip_means(ctx: PTnsCtx; srcSize, dstSize, groups: int64; src: THipMem;
  offset: int64; means: THipMem): longint; cdecl; external libtns;
function tns_hip_variances(ctx: PTnsCtx; srcSize, dstSize, groups: int64; src: THipMem;
  offset: int64; means, vars: THipMem): longint; cdecl; external libtns;
function tns_hip_normalize(ctx: PTnsCtx; srcSize, dstSize, groups: int64; means: THipMem;
  meansStride: int64; vars: THipMem; varsStride: int64; dst: THipMem; dstOffset: int64): longint;
  cdecl; external libtns;
function tns_hip_forward_scale(ctx: PTnsCtx; dstSize: int64; dst: THipMem; offset,
  scaleSize: int64; scale: THipMem; incb, batch: int64): longint; cdecl; external libtns;
function tns_hip_forward_scale_add(ctx: PTnsCtx; dstSize: int64; dst: THipMem; offset,
  scaleSize: int64; scales, biases: THipMem; incb, batch: int64): longint; cdecl; external libtns;
function tns_hip_means_and_vars_delta(ctx: PTnsCtx; srcSize, dstSize, groups: int64; delta,
  x: THipMem; offset: int64; mean, variance, mean_delta, variance_delta: THipMem): longint;
  cdecl; external libtns;
function tns_hip_normalize_delta(ctx: PTnsCtx; deltaSize, meanSize, groups: int64; delta,
  x: THipMem; offset: int64; mean, variance, mean_delta, variance_delta: THipMem): longint;
  cdecl; external libtns;
function tns_hip_add_dots(ctx: PTnsCtx; N, dstSize, groups: int64; src1, src2: THipMem;
  srcOffset: int64; dst: THipMem): longint; cdecl; external libtns;
function tns_hip_softmax_batch(ctx: PTnsCtx; N: int64; input: THipMem; iOffset, batch,
  batch_size, groups, group_size, stride: int64; temp: single; output: THipMem;
  oOffset: int64): longint; cdecl; external libtns;
function tns_hip_cross_entropy_softmax(ctx: PTnsCtx; N: int64; pred, truth, delta,
  error: THipMem): longint; cdecl; external libtns;
function tns_hip_sum(ctx: PTnsCtx; N: int64; src: THipMem; offset: int64; res: THipMem): longint;
  cdecl; external libtns;

{ fused connected-network train step (config 5) }
function tns_mlp_buffer_floats(nlayers: longint; widths: PInt64; bn: longint; batch: int64): int64;
  cdecl; external libtns;
function tns_hip_mlp_train_step(ctx: PTnsCtx; nlayers: longint; widths: PInt64; acts: PLongint;
  bn: longint; batch: int64; X, truth: THipMem; learningRate, momentum, decay: single;
  buf, cost: THipMem): longint; cdecl; external libtns;

{ layer drivers }
function tns_hip_conv2d(ctx: PTnsCtx; batch, C, H, W: int64; input, weights: THipMem;
  filters, kH, kW, wPadding, hPadding, xStride, yStride, xDilation, yDilation: int64;
  workspace, output: THipMem): longint; cdecl; external libtns;
function tns_hip_conv_forward(ctx: PTnsCtx; batch, C, H, W: int64; input, weights,
  biases: THipMem; filters, kSize, stride, padding, dilation: int64; activation: longint;
  workspace, output: THipMem; fused: longint): longint; cdecl; external libtns;
function tns_hip_conv_forward_train(ctx: PTnsCtx; batch, C, H, W: int64; input,
  weights: THipMem; filters, kSize, stride, padding, dilation: int64; activation: longint;
  scales, biases, rolling_mean, rolling_variance: THipMem; bnMomentum: single;
  training: longint; mean, variance, x, x_norm, workspace, output: THipMem): longint;
  cdecl; external libtns;
function tns_hip_conv_backward(ctx: PTnsCtx; batch, C, H, W: int64; input, weights: THipMem;
  filters, kSize, stride, padding, dilation: int64; activation: longint; output, delta,
  bias_updates, weight_updates, workspace, state_delta: THipMem): longint;
  cdecl; external libtns;
function tns_hip_conv_backward_bn(ctx: PTnsCtx; batch, C, H, W: int64; input,
  weights: THipMem; filters, kSize, stride, padding, dilation: int64; activation: longint;
  output, delta, scales, x, x_norm, mean, variance, scale_updates, mean_delta, variance_delta,
  weight_updates, workspace, state_delta: THipMem): longint; cdecl; external libtns;

{ several GPUs from one process }
function tns_hip_sgemm_strided_batched_multi(devices: PLongint; n: longint; transA,
  transB: boolean; M, N, K: int64; alpha: single; A: PSingle; lda, strideA: int64; B: PSingle;
  ldb, strideB: int64; beta: single; C: PSingle; ldc, strideC, batchCount: int64): longint;
  cdecl; external libtns;
function tns_set_op_devices(devices: PLongint; n: longint): longint; cdecl; external libtns;

{ telemetry }
function tns_hip_set_telemetry(ctx: PTnsCtx; enable: longint): longint; cdecl; external libtns;
function tns_hip_op_ms(ctx: PTnsCtx; op: longint): double; cdecl; external libtns;

{ tuning / options }
function tns_gemm_variant_count(): longint; cdecl; external libtns;
function tns_conv_dx_tile_count(): longint; cdecl; external libtns;
function tns_conv_dx_conv_count(): longint; cdecl; external libtns;
function tns_conv_dw_res_count(): longint; cdecl; external libtns;
function tns_conv_dw_tile_count(): longint; cdecl; external libtns;
function tns_conv_tile_variant_count(): longint; cdecl; external libtns;
function tns_conv_tile_variant_name(variant: longint): PAnsiChar; cdecl; external libtns;
function tns_conv_slab_count(): longint; cdecl; external libtns;
function tns_conv1x1_count(): longint; cdecl; external libtns;
function tns_conv1x1_name(variant: longint): PAnsiChar; cdecl; external libtns;
function tns_conv_slab_name(variant: longint): PAnsiChar; cdecl; external libtns;
function tns_conv_pp_variant_count(): longint; cdecl; external libtns;
function tns_conv_pp_variant_name(variant: longint): PAnsiChar; cdecl; external libtns;
function tns_conv_dma_variant_count(): longint; cdecl; external libtns;
function tns_conv_dma_variant_name(variant: longint): PAnsiChar; cdecl; external libtns;
function tns_conv_patch_variant_count(): longint; cdecl; external libtns;
function tns_conv_patch_variant_name(variant: longint): PAnsiChar; cdecl; external libtns;
function tns_sdot_chains_variant_count(): longint; cdecl; external libtns;
function tns_sdot_chains_variant_name(variant: longint): PAnsiChar; cdecl; external libtns;
function tns_sdot_rc_variant_count(): longint; cdecl; external libtns;
function tns_sdot_rc_variant_name(variant: longint): PAnsiChar; cdecl; external libtns;
function tns_gemm_variant_name(variant: longint): PAnsiChar; cdecl; external libtns;
function tns_hip_gemm_variant(ctx: PTnsCtx; variant: longint; transA, transB: boolean;
  M, N, K: int64; ALPHA: single; A: THipMem; aOffset, lda, strideA: int64; B: THipMem; bOffset,
  ldb, strideB: int64; BETA: single; C: THipMem; cOffset, ldc, strideC, batchCount: int64): longint;
  cdecl; external libtns;
function tns_set_option(opt: longint; value: int64): longint; cdecl; external libtns;

type
  { TNNHip<T>: the method list of TNNCuda<T> (nncuda.pas:100-157) over the
    HIP context.  Device buffers are TCUMem = ^T with ELEMENT offsets. }
  TNNHip<T> = class
  type
    PCUMem = ^TCUMem;
    TCUMem = ^T;
  private
    FCtx: PTnsCtx;
    procedure check(const status: longint);
    class function s(const v: T): single; static; inline;
  public
    class function deviceCount(): longint;
    constructor Create(deviceIndex: longint = 0);
    destructor Destroy(); override;
    function CompileLog: ansistring;
    function createDeviceBuffer(const N: SizeInt): TCUMem;
    procedure freeDeviceBuffer(cudaMem: TCUMem);
    procedure readBuffer(const cudaMem: TCUMem; const bufferSize: size_t; const buffer: pointer);
    procedure writeBuffer(const cudaMem: TCUMem; const bufferSize: size_t; const buffer: pointer);
    procedure ActivateArray(const N: SizeInt; const x: TCUMem; const offset: SizeInt; const activation: longint);
    procedure activateArraySWISH(const N: SizeInt; const x: TCUMem; const offset: SizeInt; const output_sigmoid, output: TCUMem);
    procedure DeriveArray(const N: SizeInt; const x: TCUMem; const offset: SizeInt; const activation: longint; delta: TCUMem);
    procedure forwardBias(const dstSize: SizeInt; const dst: TCUMem; const offset: SizeInt; const srcSize: SizeInt; const src: TCUMem; const incb: SizeInt; const batch: SizeInt);
    procedure backwardBias(const dstSize: SizeInt; const dst: TCUMem; const srcSize: SizeInt; const src: TCUMem; const srcOffset: SizeInt; const incb: SizeInt; const batch: SizeInt);
    procedure gemm(const transA, transB: boolean; const M, N, K: SizeInt; const ALPHA: T; const A: TCUMem; const aOffset: SizeInt; const lda: SizeInt; const B: TCUMem; const bOffset: SizeInt; const ldb: SizeInt; const BETA: T; const C: TCUMem; const cOffset: SizeInt; const ldc: SizeInt);
    procedure gemmBatched(const transA, transB: boolean; const M, N, K: SizeInt; const ALPHA: T; const A: PCUMem; const aOffset: SizeInt; const lda: SizeInt; const B: PCUMem; const bOffset: SizeInt; const ldb: SizeInt; const BETA: T; const C: PCUMem; const cOffset: SizeInt; const ldc: SizeInt; const batchCount: SizeInt);
    procedure gemmStridedBatched(const transA, transB: boolean; const M, N, K: SizeInt; const ALPHA: T; A: TCUMem; const aOffset: SizeInt; const lda: SizeInt; const strideA: SizeInt; B: TCUMem; const bOffset: SizeInt; const ldb: SizeInt; const strideB: SizeInt; const BETA: T; C: TCUMem; const cOffset: SizeInt; const ldc: SizeInt; const strideC: SizeInt; const batchCount: SizeInt);
    procedure addvv(const N: SizeInt; const src1: TCUMem; const src1Offset, inca: SizeInt; const src2: TCUMem; const src2Offset, incb: SizeInt; dst: TCUMem; const dstOffset, incc: SizeInt);
    procedure subvv(const N: SizeInt; const src1: TCUMem; const src1Offset, inca: SizeInt; const src2: TCUMem; const src2Offset, incb: SizeInt; dst: TCUMem; const dstOffset, incc: SizeInt);
    procedure mulvv(const N: SizeInt; const src1: TCUMem; const src1Offset, inca: SizeInt; const src2: TCUMem; const src2Offset, incb: SizeInt; dst: TCUMem; const dstOffset, incc: SizeInt);
    procedure fmavv(const N: SizeInt; const src1: TCUMem; const src1Offset, inca: SizeInt; const src2: TCUMem; const src2Offset, incb: SizeInt; const src3: TCUMem; const src3Offset, incc: SizeInt; dst: TCUMem; const dstOffset, incd: SizeInt);
    procedure axpy(const N: SizeInt; const a: T; const x: TCUMem; const xOffset: SizeInt; const incx: SizeInt; const y: TCUMem; const yOffset: SizeInt; const incy: SizeInt);
    procedure power(const N: SizeInt; const x: TCUMem; const xOffset: SizeInt; const incx: SizeInt; const a: T; const y: TCUMem; const yOffset: SizeInt; const incy: SizeInt);
    procedure scale(const N: SizeInt; const a: T; const x: TCUMem; const stride: SizeInt);
    procedure crossEntropyLogistic(const N: SizeInt; const pred, truth: TCUMem; delta, error: TCUMem);
    procedure fill(const N: SizeInt; const x: TCUMem; const offset: SizeInt; const val: T; const stride: SizeInt);
    procedure copy(const N: SizeInt; const src: TCUMem; const srcOffset, inca: SizeInt; const dst: TCUMem; const dstOffset, incb: SizeInt);
    procedure softmaxBatch(const N: SizeInt; const input: TCUMem; const iOffset: SizeInt; const batch, batch_size, groups, group_size, stride: SizeInt; const temp: T; const output: TCUMem; const oOffset: SizeInt);
    procedure crossEntropySoftmax(const N: SizeInt; const pred, truth: TCUMem; delta, error: TCUMem);
    procedure forwardMaxPool(const aBatch, outC, outH, outW: SizeInt; const input: TCUMem; const c, h, w: SizeInt; const stride_x, stride_y, padding, kernelSize: SizeInt; indexes, output: TCUMem);
    procedure backwardMaxPool(const aBatch, outC, outH, outW: SizeInt; output: TCUMem; const indexes, delta: TCUMem);
    procedure im2col(const aChannels, aHeight, aWidth, kernelHeight, kernelWidth, padHeight, padWidth, strideY, strideX, dilationY, dilationX: SizeInt; const im: TCUMem; const imOffset: SizeInt; const col: TCUMem; const colOffset: SizeInt);
    procedure col2im(const aChannels, aHeight, aWidth, kernelHeight, kernelWidth, padHeight, padWidth, strideY, strideX, dilationY, dilationX: SizeInt; const col: TCUMem; const colOffset: SizeInt; const im: TCUMem; const imOffset: SizeInt);
    procedure upSample(const aBatch, aChannels, outHeight, outWidth: SizeInt; const &in: TCUMem; const stride: SizeInt; const isForward: longint; const scale: T; const &out: TCUMem; const zeroIn: integer = 0);
    procedure fmavss(const N: SizeInt; const src: TCUMem; const offset: SizeInt; const scalar, bias: T; dst: TCUMem);
    procedure meansAndVars(const srcSize, dstSize, groups: SizeInt; const src: TCUMem; const offset: SizeInt; means, vars: TCUMem);
    procedure means(const srcSize, dstSize, groups: SizeInt; const src: TCUMem; const offset: SizeInt; means: TCUMem);
    procedure variances(const srcSize, dstSize, groups: SizeInt; const src: TCUMem; const offset: SizeInt; means, vars: TCUMem);
    procedure normalize(const srcSize, dstSize, groups: SizeInt; means: TCUMem; const meansStride: SizeInt; vars: TCUMem; const varsStride: SizeInt; dst: TCUMem; const dstOffset: SizeInt);
    procedure meansAndVarsDelta(const srcSize, dstSize, groups: SizeInt; delta, x: TCUMem; const offset: SizeInt; mean, variance, mean_delta, variance_delta: TCUMem);
    procedure normalizeDelta(const deltaSize, meanSize, groups: SizeInt; const delta, x: TCUMem; const offset: SizeInt; mean, variance, mean_delta, variance_delta: TCUMem);
    procedure addDots(const N, dstSize, groups: SizeInt; const src1, src2: TCUMem; const srcOffset: SizeInt; dst: TCUMem);
    procedure forwardScale(const dstSize: SizeInt; const dst: TCUMem; const offset: SizeInt; const scaleSize: SizeInt; const scale: TCUMem; const incb: SizeInt; const batch: SizeInt);
    procedure forwardScaleAdd(const dstSize: SizeInt; const dst: TCUMem; const offset: SizeInt; const scaleSize: SizeInt; const scales, biases: TCUMem; const incb: SizeInt; const batch: SizeInt);
    procedure forwardDropout(const N: SizeInt; const src: TCUMem; const probability, scale: T; rnd: TCUMem; dst: TCUMem);
    procedure backwardDropout(const N: SizeInt; const src: TCUMem; const probability, scale: T; const rnd: TCUMem; dst: TCUMem);
    procedure costL2(const N: SizeInt; const pred, truth, delta, error: TCUMem);
    procedure clamp(const N: SizeInt; const alpha: T; const src, dst: TCUMem; const stride: SizeInt = 1; offset: SizeInt = 0);
    procedure inverseSqrt(const N: SizeInt; const alpha: T; const src, dst: TCUMem; const stride: SizeInt = 1; offset: SizeInt = 0);
    procedure finish();
    function compileToCUBIN(const code, name: ansistring; const headers: TArray<PAnsiChar> = nil; const includeNames: TArray<PAnsiChar> = nil): RawByteString;
    procedure loadCUBIN(const cubin: RawByteString);
    function compileFile(const filename: ansistring): RawByteString;
    procedure loadCUBinFile(const filename: ansistring);

    { hot-path layer drivers beyond TNNCuda's list (tns.h "layer drivers") }
    procedure conv2D(const batch, C, H, W: SizeInt; const input, weights: TCUMem; const filters, kH, kW, wPadding, hPadding, xStride, yStride, xDilation, yDilation: SizeInt; const workspace, output: TCUMem);
    procedure convForward(const batch, C, H, W: SizeInt; const input, weights, biases: TCUMem; const filters, kSize, stride, padding, dilation: SizeInt; const activation: longint; const workspace, output: TCUMem; const fused: longint = TNS_CONV_FUSED);
    procedure convBackward(const batch, C, H, W: SizeInt; const input, weights: TCUMem; const filters, kSize, stride, padding, dilation: SizeInt; const activation: longint; const output, delta, bias_updates, weight_updates, workspace, state_delta: TCUMem);
    procedure sgdUpdate(const nWeights: SizeInt; const weights, weight_updates: TCUMem; const n: SizeInt; const biases, bias_updates, scales, scale_updates: TCUMem; const learningRate: T; const batch: SizeInt; const momentum, decay: T);

    property ctx: PTnsCtx read FCtx;
  end;

var
  hip: TNNHip<single> = nil;

{ initCUDART twin (ntensors.pas:6191-6210): one context per process, created
  once; device buffers of TTensor mirror as under USE_CUDART.  srssQuirk as
  useHipOpTable below: true (the default) selects the configured USE_AVX2
  lane drop of srss / sVarinceDelta_avx, so TNNHip.variances /
  meansAndVarsDelta reproduce the CPU build's batch-norm statistics.
  pipelineBackward = true (the default) sets TNS_OPT_BWD_OVERLAP = 2: each
  convBackward call (TConvolutionalLayer.backwardGPU, in TNet.backward's
  loop nnet.pas:332-366) leaves its dW product running on the context's side
  stream under the following layers' work; the next call of any other
  TNNHip method (sgdUpdate in TNet.update, readBuffer, finish, a non-conv
  layer's backward) joins it first, so every access made through TNNHip
  sees finished weight_updates.  Contract (include/tns.h): nothing may read
  or write a pending layer's weight_updates, or write its input or delta,
  outside this API before such a join.  false keeps the library default
  (1: dW and state.delta concurrently, joined before each call returns). }
procedure initHIP(const deviceIndex: SizeInt; const srssQuirk: boolean = true;
  const pipelineBackward: boolean = true);

{ Bind the host-pointer op-table drop-ins (boundary A) after
  TTensorOps.initSingle, as USE_OPENBLAS / USE_MKL do (ntensors.pas:
  12735-12756):
      TSingleTensor.gemm := @tns_cblas_sgemm; ...
  srssQuirk = true sets TNS_OPT_SRSS_QUIRK = 1 so the GPU MeansAndVars /
  sMeanAndVarianceDelta drop lanes 4..7 of blocks that are a multiple of 8
  long, exactly as the reference's configured USE_AVX2 srss /
  sVarinceDelta_avx do (ntensors.pas:1509-1511, 8739-8741; every YOLOv3
  conv block at 52^2 and above).  The library default (false) folds those
  lanes back in (the mathematically intended variance); a drop-in that must
  reproduce the CPU build's numbers passes true. }
procedure useHipOpTable(const srssQuirk: boolean = true);

implementation

{ ---- TNNHip<T> ------------------------------------------------------------ }

procedure TNNHip<T>.check(const status: longint);
begin
  if status <> TNS_OK then
    raise ETnsError.CreateFmt('tensorium_hip: status %d: %s', [status, string(tns_last_error())]);
end;

class function TNNHip<T>.s(const v: T): single;
begin
  result := PSingle(@v)^
end;

class function TNNHip<T>.deviceCount(): longint;
begin
  result := tns_device_count()
end;

constructor TNNHip<T>.Create(deviceIndex: longint);
begin
  if SizeOf(T) <> SizeOf(single) then
    raise ENotSupportedException.Create('TNNHip: the MI355X backend computes fp32 only');
  check(tns_hip_create(deviceIndex, @FCtx));
end;

destructor TNNHip<T>.Destroy();
begin
  if assigned(FCtx) then
    tns_hip_destroy(FCtx);
  FCtx := nil;
  inherited Destroy
end;

function TNNHip<T>.CompileLog: ansistring;
begin
  result := ''      { kernels are compiled ahead of time for gfx950 }
end;

function TNNHip<T>.createDeviceBuffer(const N: SizeInt): TCUMem;
var p: THipMem;
begin
  check(tns_hip_malloc(FCtx, N, @p));
  result := TCUMem(p)
end;

procedure TNNHip<T>.freeDeviceBuffer(cudaMem: TCUMem);
begin
  check(tns_hip_free(FCtx, THipMem(cudaMem)))
end;

procedure TNNHip<T>.readBuffer(const cudaMem: TCUMem; const bufferSize: size_t; const buffer: pointer);
begin
  check(tns_hip_read_buffer(FCtx, THipMem(cudaMem), bufferSize, buffer))
end;

procedure TNNHip<T>.writeBuffer(const cudaMem: TCUMem; const bufferSize: size_t; const buffer: pointer);
begin
  check(tns_hip_write_buffer(FCtx, THipMem(cudaMem), bufferSize, buffer))
end;

procedure TNNHip<T>.ActivateArray(const N: SizeInt; const x: TCUMem; const offset: SizeInt; const activation: longint);
begin
  check(tns_hip_activate_array(FCtx, N, THipMem(x), offset, activation))
end;

procedure TNNHip<T>.activateArraySWISH(const N: SizeInt; const x: TCUMem; const offset: SizeInt; const output_sigmoid, output: TCUMem);
begin
  raise ENotSupportedException.Create('TNNHip.activateArraySWISH: not on the hot path (SURVEY.md §8)')
end;

procedure TNNHip<T>.DeriveArray(const N: SizeInt; const x: TCUMem; const offset: SizeInt; const activation: longint; delta: TCUMem);
begin
  check(tns_hip_derive_array(FCtx, N, THipMem(x), offset, activation, THipMem(delta)))
end;

procedure TNNHip<T>.forwardBias(const dstSize: SizeInt; const dst: TCUMem; const offset: SizeInt; const srcSize: SizeInt; const src: TCUMem; const incb: SizeInt; const batch: SizeInt);
begin
  check(tns_hip_forward_bias(FCtx, dstSize, THipMem(dst), offset, srcSize, THipMem(src), incb, batch))
end;

procedure TNNHip<T>.backwardBias(const dstSize: SizeInt; const dst: TCUMem; const srcSize: SizeInt; const src: TCUMem; const srcOffset: SizeInt; const incb: SizeInt; const batch: SizeInt);
begin
  check(tns_hip_backward_bias(FCtx, dstSize, THipMem(dst), srcSize, THipMem(src), srcOffset, incb, batch))
end;

procedure TNNHip<T>.gemm(const transA, transB: boolean; const M, N, K: SizeInt; const ALPHA: T; const A: TCUMem; const aOffset: SizeInt; const lda: SizeInt; const B: TCUMem; const bOffset: SizeInt; const ldb: SizeInt; const BETA: T; const C: TCUMem; const cOffset: SizeInt; const ldc: SizeInt);
begin
  check(tns_hip_gemm(FCtx, transA, transB, M, N, K, s(ALPHA), THipMem(A), aOffset, lda,
    THipMem(B), bOffset, ldb, s(BETA), THipMem(C), cOffset, ldc))
end;

procedure TNNHip<T>.gemmBatched(const transA, transB: boolean; const M, N, K: SizeInt; const ALPHA: T; const A: PCUMem; const aOffset: SizeInt; const lda: SizeInt; const B: PCUMem; const bOffset: SizeInt; const ldb: SizeInt; const BETA: T; const C: PCUMem; const cOffset: SizeInt; const ldc: SizeInt; const batchCount: SizeInt);
begin
  { A, B, C: arrays of device pointers, device-resident as the reference
    builds them with writeBuffer (nConvolutionLayer.pas:1083-1085) for
    cublasSgemmBatched_64 (nncuda.pas:752); the library reads them in stream
    order }
  check(tns_hip_gemm_batched(FCtx, transA, transB, M, N, K, s(ALPHA), PHipMem(A), aOffset, lda,
    PHipMem(B), bOffset, ldb, s(BETA), PHipMem(C), cOffset, ldc, batchCount))
end;

procedure TNNHip<T>.gemmStridedBatched(const transA, transB: boolean; const M, N, K: SizeInt; const ALPHA: T; A: TCUMem; const aOffset: SizeInt; const lda: SizeInt; const strideA: SizeInt; B: TCUMem; const bOffset: SizeInt; const ldb: SizeInt; const strideB: SizeInt; const BETA: T; C: TCUMem; const cOffset: SizeInt; const ldc: SizeInt; const strideC: SizeInt; const batchCount: SizeInt);
begin
  check(tns_hip_gemm_strided_batched(FCtx, transA, transB, M, N, K, s(ALPHA), THipMem(A), aOffset,
    lda, strideA, THipMem(B), bOffset, ldb, strideB, s(BETA), THipMem(C), cOffset, ldc, strideC,
    batchCount))
end;

procedure TNNHip<T>.addvv(const N: SizeInt; const src1: TCUMem; const src1Offset, inca: SizeInt; const src2: TCUMem; const src2Offset, incb: SizeInt; dst: TCUMem; const dstOffset, incc: SizeInt);
begin
  check(tns_hip_addvv(FCtx, N, THipMem(src1), src1Offset, inca, THipMem(src2), src2Offset, incb,
    THipMem(dst), dstOffset, incc))
end;

procedure TNNHip<T>.subvv(const N: SizeInt; const src1: TCUMem; const src1Offset, inca: SizeInt; const src2: TCUMem; const src2Offset, incb: SizeInt; dst: TCUMem; const dstOffset, incc: SizeInt);
begin
  check(tns_hip_subvv(FCtx, N, THipMem(src1), src1Offset, inca, THipMem(src2), src2Offset, incb,
    THipMem(dst), dstOffset, incc))
end;

procedure TNNHip<T>.mulvv(const N: SizeInt; const src1: TCUMem; const src1Offset, inca: SizeInt; const src2: TCUMem; const src2Offset, incb: SizeInt; dst: TCUMem; const dstOffset, incc: SizeInt);
begin
  check(tns_hip_mulvv(FCtx, N, THipMem(src1), src1Offset, inca, THipMem(src2), src2Offset, incb,
    THipMem(dst), dstOffset, incc))
end;

procedure TNNHip<T>.fmavv(const N: SizeInt; const src1: TCUMem; const src1Offset, inca: SizeInt; const src2: TCUMem; const src2Offset, incb: SizeInt; const src3: TCUMem; const src3Offset, incc: SizeInt; dst: TCUMem; const dstOffset, incd: SizeInt);
begin
  check(tns_hip_fmavv(FCtx, N, THipMem(src1), src1Offset, inca, THipMem(src2), src2Offset, incb,
    THipMem(src3), src3Offset, incc, THipMem(dst), dstOffset, incd))
end;

procedure TNNHip<T>.axpy(const N: SizeInt; const a: T; const x: TCUMem; const xOffset: SizeInt; const incx: SizeInt; const y: TCUMem; const yOffset: SizeInt; const incy: SizeInt);
begin
  check(tns_hip_axpy(FCtx, N, s(a), THipMem(x), xOffset, incx, THipMem(y), yOffset, incy))
end;

procedure TNNHip<T>.power(const N: SizeInt; const x: TCUMem; const xOffset: SizeInt; const incx: SizeInt; const a: T; const y: TCUMem; const yOffset: SizeInt; const incy: SizeInt);
begin
  raise ENotSupportedException.Create('TNNHip.power: not on the hot path (SURVEY.md §8)')
end;

procedure TNNHip<T>.scale(const N: SizeInt; const a: T; const x: TCUMem; const stride: SizeInt);
begin
  check(tns_hip_scale(FCtx, N, s(a), THipMem(x), stride))
end;

procedure TNNHip<T>.crossEntropyLogistic(const N: SizeInt; const pred, truth: TCUMem; delta, error: TCUMem);
begin
  raise ENotSupportedException.Create('TNNHip.crossEntropyLogistic: not on the hot path (SURVEY.md §8)')
end;

procedure TNNHip<T>.fill(const N: SizeInt; const x: TCUMem; const offset: SizeInt; const val: T; const stride: SizeInt);
begin
  check(tns_hip_fill(FCtx, N, THipMem(x), offset, s(val), stride))
end;

procedure TNNHip<T>.copy(const N: SizeInt; const src: TCUMem; const srcOffset, inca: SizeInt; const dst: TCUMem; const dstOffset, incb: SizeInt);
begin
  check(tns_hip_copy(FCtx, N, THipMem(src), srcOffset, inca, THipMem(dst), dstOffset, incb))
end;

procedure TNNHip<T>.softmaxBatch(const N: SizeInt; const input: TCUMem; const iOffset: SizeInt; const batch, batch_size, groups, group_size, stride: SizeInt; const temp: T; const output: TCUMem; const oOffset: SizeInt);
begin
  check(tns_hip_softmax_batch(FCtx, N, THipMem(input), iOffset, batch, batch_size, groups,
    group_size, stride, s(temp), THipMem(output), oOffset))
end;

procedure TNNHip<T>.crossEntropySoftmax(const N: SizeInt; const pred, truth: TCUMem; delta, error: TCUMem);
begin
  check(tns_hip_cross_entropy_softmax(FCtx, N, THipMem(pred), THipMem(truth), THipMem(delta),
    THipMem(error)))
end;

procedure TNNHip<T>.forwardMaxPool(const aBatch, outC, outH, outW: SizeInt; const input: TCUMem; const c, h, w: SizeInt; const stride_x, stride_y, padding, kernelSize: SizeInt; indexes, output: TCUMem);
begin
  raise ENotSupportedException.Create('TNNHip.forwardMaxPool: not on the hot path (SURVEY.md §8)')
end;

procedure TNNHip<T>.backwardMaxPool(const aBatch, outC, outH, outW: SizeInt; output: TCUMem; const indexes, delta: TCUMem);
begin
  raise ENotSupportedException.Create('TNNHip.backwardMaxPool: not on the hot path (SURVEY.md §8)')
end;

procedure TNNHip<T>.im2col(const aChannels, aHeight, aWidth, kernelHeight, kernelWidth, padHeight, padWidth, strideY, strideX, dilationY, dilationX: SizeInt; const im: TCUMem; const imOffset: SizeInt; const col: TCUMem; const colOffset: SizeInt);
begin
  check(tns_hip_im2col(FCtx, aChannels, aHeight, aWidth, kernelHeight, kernelWidth, padHeight,
    padWidth, strideY, strideX, dilationY, dilationX, THipMem(im), imOffset, THipMem(col), colOffset))
end;

procedure TNNHip<T>.col2im(const aChannels, aHeight, aWidth, kernelHeight, kernelWidth, padHeight, padWidth, strideY, strideX, dilationY, dilationX: SizeInt; const col: TCUMem; const colOffset: SizeInt; const im: TCUMem; const imOffset: SizeInt);
begin
  check(tns_hip_col2im(FCtx, aChannels, aHeight, aWidth, kernelHeight, kernelWidth, padHeight,
    padWidth, strideY, strideX, dilationY, dilationX, THipMem(col), colOffset, THipMem(im), imOffset))
end;

procedure TNNHip<T>.upSample(const aBatch, aChannels, outHeight, outWidth: SizeInt; const &in: TCUMem; const stride: SizeInt; const isForward: longint; const scale: T; const &out: TCUMem; const zeroIn: integer);
begin
  check(tns_hip_upsample(FCtx, aBatch, aChannels, outHeight, outWidth, THipMem(&in), stride,
    isForward, s(scale), THipMem(&out), zeroIn))
end;

procedure TNNHip<T>.fmavss(const N: SizeInt; const src: TCUMem; const offset: SizeInt; const scalar, bias: T; dst: TCUMem);
begin
  check(tns_hip_fmavss(FCtx, N, THipMem(src), offset, s(scalar), s(bias), THipMem(dst)))
end;

procedure TNNHip<T>.meansAndVars(const srcSize, dstSize, groups: SizeInt; const src: TCUMem; const offset: SizeInt; means, vars: TCUMem);
begin
  check(tns_hip_means_and_vars(FCtx, srcSize, dstSize, groups, THipMem(src), offset,
    THipMem(means), THipMem(vars)))
end;

procedure TNNHip<T>.means(const srcSize, dstSize, groups: SizeInt; const src: TCUMem; const offset: SizeInt; means: TCUMem);
begin
  { batchNormGPU (nbaselayer.pas:583), TConnectedLayer.forwardGPU
    (nconnectedlayer.pas:664): MeansAndVars' mean (vssum_avx2 lanes) }
  check(tns_hip_means(FCtx, srcSize, dstSize, groups, THipMem(src), offset, THipMem(means)))
end;

procedure TNNHip<T>.variances(const srcSize, dstSize, groups: SizeInt; const src: TCUMem; const offset: SizeInt; means, vars: TCUMem);
begin
  { batchNormGPU (nbaselayer.pas:584): the unbiased variance about the given
    means in MeansAndVars' srss order (TNS_OPT_SRSS_QUIRK as set by initHIP) }
  check(tns_hip_variances(FCtx, srcSize, dstSize, groups, THipMem(src), offset, THipMem(means),
    THipMem(vars)))
end;

procedure TNNHip<T>.normalize(const srcSize, dstSize, groups: SizeInt; means: TCUMem; const meansStride: SizeInt; vars: TCUMem; const varsStride: SizeInt; dst: TCUMem; const dstOffset: SizeInt);
begin
  check(tns_hip_normalize(FCtx, srcSize, dstSize, groups, THipMem(means), meansStride,
    THipMem(vars), varsStride, THipMem(dst), dstOffset))
end;

procedure TNNHip<T>.meansAndVarsDelta(const srcSize, dstSize, groups: SizeInt; delta, x: TCUMem; const offset: SizeInt; mean, variance, mean_delta, variance_delta: TCUMem);
begin
  check(tns_hip_means_and_vars_delta(FCtx, srcSize, dstSize, groups, THipMem(delta), THipMem(x),
    offset, THipMem(mean), THipMem(variance), THipMem(mean_delta), THipMem(variance_delta)))
end;

procedure TNNHip<T>.normalizeDelta(const deltaSize, meanSize, groups: SizeInt; const delta, x: TCUMem; const offset: SizeInt; mean, variance, mean_delta, variance_delta: TCUMem);
begin
  check(tns_hip_normalize_delta(FCtx, deltaSize, meanSize, groups, THipMem(delta), THipMem(x),
    offset, THipMem(mean), THipMem(variance), THipMem(mean_delta), THipMem(variance_delta)))
end;

procedure TNNHip<T>.addDots(const N, dstSize, groups: SizeInt; const src1, src2: TCUMem; const srcOffset: SizeInt; dst: TCUMem);
begin
  check(tns_hip_add_dots(FCtx, N, dstSize, groups, THipMem(src1), THipMem(src2), srcOffset,
    THipMem(dst)))
end;

procedure TNNHip<T>.forwardScale(const dstSize: SizeInt; const dst: TCUMem; const offset: SizeInt; const scaleSize: SizeInt; const scale: TCUMem; const incb: SizeInt; const batch: SizeInt);
begin
  check(tns_hip_forward_scale(FCtx, dstSize, THipMem(dst), offset, scaleSize, THipMem(scale),
    incb, batch))
end;

procedure TNNHip<T>.forwardScaleAdd(const dstSize: SizeInt; const dst: TCUMem; const offset: SizeInt; const scaleSize: SizeInt; const scales, biases: TCUMem; const incb: SizeInt; const batch: SizeInt);
begin
  check(tns_hip_forward_scale_add(FCtx, dstSize, THipMem(dst), offset, scaleSize,
    THipMem(scales), THipMem(biases), incb, batch))
end;

procedure TNNHip<T>.forwardDropout(const N: SizeInt; const src: TCUMem; const probability, scale: T; rnd: TCUMem; dst: TCUMem);
begin
  raise ENotSupportedException.Create('TNNHip.forwardDropout: not on the hot path (SURVEY.md §8)')
end;

procedure TNNHip<T>.backwardDropout(const N: SizeInt; const src: TCUMem; const probability, scale: T; const rnd: TCUMem; dst: TCUMem);
begin
  raise ENotSupportedException.Create('TNNHip.backwardDropout: not on the hot path (SURVEY.md §8)')
end;

procedure TNNHip<T>.costL2(const N: SizeInt; const pred, truth, delta, error: TCUMem);
begin
  raise ENotSupportedException.Create('TNNHip.costL2: not on the hot path (SURVEY.md §8)')
end;

procedure TNNHip<T>.clamp(const N: SizeInt; const alpha: T; const src, dst: TCUMem; const stride: SizeInt; offset: SizeInt);
begin
  check(tns_hip_clamp(FCtx, N, s(alpha), THipMem(src), THipMem(dst), stride, offset))
end;

procedure TNNHip<T>.inverseSqrt(const N: SizeInt; const alpha: T; const src, dst: TCUMem; const stride: SizeInt; offset: SizeInt);
begin
  check(tns_hip_inverse_sqrt(FCtx, N, s(alpha), THipMem(src), THipMem(dst), stride, offset))
end;

procedure TNNHip<T>.finish();
begin
  check(tns_hip_finish(FCtx))
end;

function TNNHip<T>.compileToCUBIN(const code, name: ansistring; const headers: TArray<PAnsiChar>; const includeNames: TArray<PAnsiChar>): RawByteString;
begin
  raise ENotSupportedException.Create('TNNHip: kernels are built ahead of time for gfx950 (no runtime compilation)')
end;

procedure TNNHip<T>.loadCUBIN(const cubin: RawByteString);
begin
  raise ENotSupportedException.Create('TNNHip: kernels are built ahead of time for gfx950 (no runtime compilation)')
end;

function TNNHip<T>.compileFile(const filename: ansistring): RawByteString;
begin
  raise ENotSupportedException.Create('TNNHip: kernels are built ahead of time for gfx950 (no runtime compilation)')
end;

procedure TNNHip<T>.loadCUBinFile(const filename: ansistring);
begin
  raise ENotSupportedException.Create('TNNHip: kernels are built ahead of time for gfx950 (no runtime compilation)')
end;

procedure TNNHip<T>.conv2D(const batch, C, H, W: SizeInt; const input, weights: TCUMem; const filters, kH, kW, wPadding, hPadding, xStride, yStride, xDilation, yDilation: SizeInt; const workspace, output: TCUMem);
begin
  check(tns_hip_conv2d(FCtx, batch, C, H, W, THipMem(input), THipMem(weights), filters, kH, kW,
    wPadding, hPadding, xStride, yStride, xDilation, yDilation, THipMem(workspace), THipMem(output)))
end;

procedure TNNHip<T>.convForward(const batch, C, H, W: SizeInt; const input, weights, biases: TCUMem; const filters, kSize, stride, padding, dilation: SizeInt; const activation: longint; const workspace, output: TCUMem; const fused: longint);
begin
  check(tns_hip_conv_forward(FCtx, batch, C, H, W, THipMem(input), THipMem(weights),
    THipMem(biases), filters, kSize, stride, padding, dilation, activation, THipMem(workspace),
    THipMem(output), fused))
end;

procedure TNNHip<T>.convBackward(const batch, C, H, W: SizeInt; const input, weights: TCUMem; const filters, kSize, stride, padding, dilation: SizeInt; const activation: longint; const output, delta, bias_updates, weight_updates, workspace, state_delta: TCUMem);
begin
  check(tns_hip_conv_backward(FCtx, batch, C, H, W, THipMem(input), THipMem(weights), filters,
    kSize, stride, padding, dilation, activation, THipMem(output), THipMem(delta),
    THipMem(bias_updates), THipMem(weight_updates), THipMem(workspace), THipMem(state_delta)))
end;

procedure TNNHip<T>.sgdUpdate(const nWeights: SizeInt; const weights, weight_updates: TCUMem; const n: SizeInt; const biases, bias_updates, scales, scale_updates: TCUMem; const learningRate: T; const batch: SizeInt; const momentum, decay: T);
var lrb, ndb: single;
begin
  { args.learningRate / args.batch and -args.decay * args.batch in single,
    as TConnectedLayer.update (nconnectedlayer.pas:332, 347) }
  lrb := s(learningRate) / batch;
  ndb := -s(decay) * batch;
  check(tns_hip_sgd_update(FCtx, nWeights, THipMem(weights), THipMem(weight_updates), n,
    THipMem(biases), THipMem(bias_updates), THipMem(scales), THipMem(scale_updates), lrb, ndb,
    s(momentum)))
end;

{ ---- process-wide setup ---------------------------------------------------- }

procedure initHIP(const deviceIndex: SizeInt; const srssQuirk: boolean;
  const pipelineBackward: boolean);
begin
  if srssQuirk then
    tns_set_option(TNS_OPT_SRSS_QUIRK, 1)
  else
    tns_set_option(TNS_OPT_SRSS_QUIRK, 0);
  if pipelineBackward then
    tns_set_option(TNS_OPT_BWD_OVERLAP, 2)
  else
    tns_set_option(TNS_OPT_BWD_OVERLAP, 1);
  if not assigned(hip) then
    hip := TNNHip<single>.Create(deviceIndex)
end;

procedure hipFatal(code: longint; msg: PAnsiChar); cdecl;
begin
  { the op-table pointer types carry no status: fail loudly, as SAFE_CALL }
  raise ETnsError.CreateFmt('tensorium_hip op-table call failed (%d): %s', [code, string(msg)])
end;

procedure useHipOpTable(const srssQuirk: boolean);
begin
  if tns_abi_version() <> 1 then
    raise ETnsError.Create('tensorium_hip: unexpected ABI version');
  tns_set_error_hook(@hipFatal);
  if srssQuirk then
    tns_set_option(TNS_OPT_SRSS_QUIRK, 1)
  else
    tns_set_option(TNS_OPT_SRSS_QUIRK, 0);
  { In the host unit, after TTensorOps.initSingle (ntensors.pas:12651-12758):
      TSingleTensor.gemm                   := @tns_cblas_sgemm;
      TSingleTensor.gemmStridedBatched     := @tns_cblas_sgemm_batch_strided;
      TSingleTensor.im2Colvv               := @tns_im2col;
      TSingleTensor.col2imvv               := @tns_col2im;
      TSingleTensor.im2colStridedBatchedvv := @tns_im2col_strided_batched;
      TSingleTensor.col2imStridedBatchedvv := @tns_col2im_strided_batched;
    (ntensors is not a dependency of this unit, so the assignments live in
    the caller; the parameter lists match the class-var pointer types
    exactly: INTEGRATION.md §1.) }
end;

finalization
  FreeAndNil(hip);
end.
