// `extract <file.compressed>` -> ./DECOMPRESSED_FILE, the reference decoder CLI
// (Decompressor.cu:47-114) with the decode on the gfx950 kernels of
// libhuffman_amd. Exit codes follow the reference: 1 on usage error, 0 on a
// missing file (Decompressor.cu:51-63); 2 when the codec or any other I/O fails.
#include <iostream>

#include "huffman_amd.h"

int main(int argc, char* argv[]) {
    if (argc != 2) {
        std::cout << "Missing compressed file name." << std::endl
                  << "Usage: './extract <compressed_file_name>'" << std::endl;
        return 1;
    }
    const int rc = hz_extract_file(argv[1], nullptr, 0, 1);
    if (rc == HZ_ENOENT || rc == HZ_OK) return 0;
    return 2;
}
