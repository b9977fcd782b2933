// Host-only driver for the AddressSanitizer build of the PLY reader (csrc/ply_loader.hip).
// Built by tests/test_ply_asan.py with `-Xarch_host -fsanitize=address`; loads every file
// named on the command line through gsr_ply_probe + gsr_ply_load (host output) and prints
// "<rc> <P>" per file.  Malformed files must come back as GSR_E_INVALID, never as a crash or
// an ASan report.  No GPU: the host-output path makes no HIP call.
#include <cstdio>
#include <string>
#include <vector>

#include "gsr.h"

static std::string g_msg;
int gsr_set_error(int code, const std::string &msg) {  // api.hip's, for this driver alone
    g_msg = msg;
    return code;
}

int main(int argc, char **argv) {
    for (int i = 1; i < argc; ++i) {
        gsr_ply_info info{};
        int rc = gsr_ply_probe(argv[i], &info);
        if (rc == 0 && info.P >= 0 && info.P <= (1 << 20)) {
            const size_t P = (size_t)info.P;
            std::vector<float> xyz(3 * P + 1), rot(4 * P + 1), scale(3 * P + 1), op(P + 1),
                sh(48 * P + 1);
            rc = gsr_ply_load(argv[i], &info, xyz.data(), rot.data(), scale.data(), op.data(),
                              sh.data(), 0, nullptr);
        }
        std::printf("%d %lld %s\n", rc, (long long)info.P, rc ? g_msg.c_str() : "");
    }
    return 0;
}
