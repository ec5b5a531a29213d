// `archive <file>` -> <file>.compressed, the reference's GPU encoder CLI
// (Compressor.cu:315-632) on the gfx950 kernels of libhuffman_amd.
// Exit codes follow the reference: 0 on usage error and on a missing file
// (Compressor.cu:317-330); 2 when the codec or any other I/O fails.
#include <iostream>

#include "huffman_amd.h"

int main(int argc, char* argv[]) {
    if (argc != 2) {
        std::cout << "Must provide a single file name." << std::endl;
        return 0;
    }
    const int rc = hz_archive_file(argv[1], 1);
    if (rc == HZ_ENOENT || rc == HZ_OK) return 0;
    return 2;
}
