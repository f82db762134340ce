// utils.cpp -- argv, directory-name and raw .bin file handling of the CLI.
// Behaviour of detker/CUDA-Flash-Attention src/utils.cpp:5-100: raw little-endian
// fp32 files with no header, a short read/write or missing file exits through ERR,
// the shape comes from the directory basename "B%d_H%d_S%d_D%d" (trailing '/'
// ignored), argv is <naive|fa1|fa2> <forward|backward|forward_backward> <fp16|fp32|bf16> <dir>.
#include <sys/stat.h>

#include <cstdio>
#include <cstring>

#include "utils.h"

bool file_exists(const char* filename) {
    struct stat st;
    return stat(filename, &st) == 0;
}

void load_binary_file(const char* filename, float* data, size_t count) {
    FILE* f = fopen(filename, "rb");
    if (!f) ERR("fopen");
    const size_t got = fread(data, sizeof(float), count, f);
    fclose(f);
    if (got != count) ERR("fread");
}

void save_binary_file(const char* filename, const float* data, size_t count) {
    FILE* f = fopen(filename, "wb");
    if (!f) ERR("fopen");
    const size_t put = fwrite(data, sizeof(float), count, f);
    fclose(f);
    if (put != count) ERR("fwrite");
}

void parse_config_string(const char* path, int* batch_size, int* num_heads, int* seq_len, int* head_dim) {
    size_t end = strlen(path);
    while (end > 0 && path[end - 1] == '/') --end;
    size_t start = end;
    while (start > 0 && path[start - 1] != '/') --start;
    char name[512];
    const size_t n = end - start < sizeof(name) - 1 ? end - start : sizeof(name) - 1;
    memcpy(name, path + start, n);
    name[n] = '\0';
    if (sscanf(name, "B%d_H%d_S%d_D%d", batch_size, num_heads, seq_len, head_dim) != 4) ERR("sscanf");
}

void parse_args(int argc, char** argv, ComputeDataType* precision, ComputeType* method, ModeType* mode,
                char** data_path) {
    if (argc < 5) usage(argv[0]);
    if (!strcmp(argv[1], "fa2")) *method = ComputeType::FlashAttention2;
    else if (!strcmp(argv[1], "fa1")) *method = ComputeType::FlashAttention1;
    else if (!strcmp(argv[1], "naive")) *method = ComputeType::Naive;
    else usage(argv[0]);

    if (!strcmp(argv[2], "forward")) *mode = ModeType::Forward;
    else if (!strcmp(argv[2], "backward")) *mode = ModeType::Backward;
    else if (!strcmp(argv[2], "forward_backward")) *mode = ModeType::ForwardBackward;
    else usage(argv[0]);

    if (!strcmp(argv[3], "fp16")) *precision = ComputeDataType::FP16;
    else if (!strcmp(argv[3], "fp32")) *precision = ComputeDataType::FP32;
    else if (!strcmp(argv[3], "bf16")) *precision = ComputeDataType::BF16;
    else usage(argv[0]);

    *data_path = argv[4];
}
