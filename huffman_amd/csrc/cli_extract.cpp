// `extract <file.compressed>` -> ./DECOMPRESSED_FILE, the reference decoder CLI
// (Decompressor.cu:47-114) with the decode on the gfx950 kernels of
// libhuffman_amd. Exit codes follow the reference: 1 on usage error, 0 on a
// missing file (Decompressor.cu:51-63); 2 when the codec or any other I/O fails.
#include <stdio.h>
#include <stdlib.h>

#include <iostream>

#include "huffman_amd.h"

int main(int argc, char* argv[]) {
    if (argc != 2) {
        std::cout << "Missing compressed file name." << std::endl
                  << "Usage: './extract <compressed_file_name>'" << std::endl;
        return 1;
    }
    const int rc = hz_extract_file(argv[1], nullptr, 0, 1);
    if (getenv("HZ_TIMING")) {  // stage split of the run, one JSON line on stderr
        hz_stream_timing t;
        if (hz_stream_last_timing(&t) == HZ_OK)
            fprintf(stderr,
                    "{\"total_ms\": %.3f, \"fread_ms\": %.3f, \"fwrite_ms\": %.3f, \"alloc_ms\": %.3f, "
                    "\"host_ms\": %.3f, "
                    "\"h2d_ms\": %.3f, \"kernel_ms\": %.3f, \"d2h_ms\": %.3f, \"bytes_in\": %llu, "
                    "\"bytes_out\": %llu}\n",
                    t.total_ms, t.fread_ms, t.fwrite_ms, t.alloc_ms, t.host_ms, t.h2d_ms, t.kernel_ms, t.d2h_ms,
                    (unsigned long long)t.bytes_in, (unsigned long long)t.bytes_out);
    }
    if (rc == HZ_ENOENT || rc == HZ_OK) return 0;
    return 2;
}
