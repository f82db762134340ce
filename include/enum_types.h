// enum_types.h -- same enums as detker/CUDA-Flash-Attention include/enum_types.h:3-18.
#pragma once

enum class ComputeType {
    Naive,            // vanilla attention (reference baseline; not built here)
    FlashAttention1,  // FA1 (reference baseline; not built here)
    FlashAttention2   // FA2 -- the hot path
};

enum class ModeType {
    Forward,
    Backward,
    ForwardBackward
};

// Precision of the on-chip (LDS/VGPR) tiles; HBM I/O is fp32 either way.
enum class ComputeDataType {
    FP16,  // fp16 tiles, MFMA f16 -> fp32 accumulate
    FP32,  // fp32 tiles, exact-fp32 MFMA
    BF16   // bf16 tiles, MFMA bf16 -> fp32 accumulate (extension: README.md:504-508)
};
