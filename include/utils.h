// utils.h -- CLI helpers with the signatures of detker/CUDA-Flash-Attention include/utils.h:9-13.
#pragma once

#include <cstddef>

#include "enum_types.h"
#include "error_utils.h"

bool file_exists(const char* filename);
void load_binary_file(const char* filename, float* data, size_t count);
void save_binary_file(const char* filename, const float* data, size_t count);
void parse_config_string(const char* path, int* batch_size, int* num_heads, int* seq_len, int* head_dim);
void parse_args(int argc, char** argv, ComputeDataType* precision, ComputeType* method, ModeType* mode,
                char** data_path);
