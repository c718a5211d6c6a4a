// Host-side AddressSanitizer driver for csrc/gridbin.hip (no GPU needed):
// the scratch query and the binned backward's argument checks and plan
// building, with the reference grid's offsets, every group / walk form /
// option combination, NULL and non-NULL options, bad arguments.
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <vector>

#include "dfhip.h"

static std::vector<int32_t> reference_offsets(uint32_t L) {
    // grid.py:110-124: res_l = ceil(16 * s^l), rows = min(2^16, (res + 1)^3) rounded up to 8
    std::vector<int32_t> off(L + 1, 0);
    const double s = std::exp2(std::log2(2048.0 / 16.0) / 15.0);
    for (uint32_t l = 0; l < L; ++l) {
        const double res = std::ceil(16.0 * std::pow(s, (double)l));
        double rows = std::pow(res + 1.0, 3.0);
        if (rows > 65536.0) rows = 65536.0;
        off[l + 1] = off[l] + (int32_t)(std::ceil(rows / 8.0) * 8.0);
    }
    return off;
}

int main() {
    int failures = 0;
    auto expect = [&](bool ok, const char *what) {
        if (!ok) {
            std::printf("FAIL %s: %s\n", what, dfhip_last_error());
            ++failures;
        }
    };
    for (uint32_t L : {1u, 2u, 16u, 24u}) {
        const std::vector<int32_t> off = reference_offsets(L);
        for (uint32_t group : {1u, 7u}) {
            for (int mode : {-1, 0, 1}) {
                for (int wg : {0, 1, 3, 16}) {
                    dfhip_binned_opts o{mode, -1, wg, -1, nullptr};
                    for (const dfhip_binned_opts *op : {(const dfhip_binned_opts *)nullptr,
                                                        (const dfhip_binned_opts *)&o}) {
                        for (uint32_t cap : {0u, 1u, 1023u, 1024u, 1u << 22}) {
                            uint64_t e = 0, c = 0, p = 0;
                            const int rc = dfhip_grid_backward_binned_scratch_opts(
                                cap, off.data(), L, 2, group, op, &e, &c, &p);
                            expect(rc == DFHIP_OK && e && c && p, "scratch query");
                            // the launch's host part: empty batch, every phase
                            // (no device pointers are dereferenced on the host)
                            for (int phase : {1, 2, 3}) {
                                (void)dfhip_grid_encode_backward_binned_opts(
                                    phase, DFHIP_F16, nullptr, nullptr, 1.0f, (const int32_t *)1,
                                    off.data(), (float *)1, 0, nullptr, 3, 2, L, 0.5f, 16, 1, 0,
                                    group, 0.01f, (uint32_t *)1, (uint32_t *)1, (float *)1, 0, op,
                                    nullptr);
                            }
                        }
                    }
                }
            }
        }
        uint64_t e, c, p;
        dfhip_binned_opts bad{2, -1, 0, -1, nullptr};
        expect(dfhip_grid_backward_binned_scratch_opts(64, off.data(), L, 2, 1, &bad, &e, &c, &p) ==
                   DFHIP_EINVAL, "walk_mode 2 rejected");
        expect(dfhip_grid_backward_binned_scratch_opts(64, off.data(), L, 2, 3, nullptr, &e, &c,
                                                       &p) == DFHIP_EINVAL, "group 3 rejected");
        expect(dfhip_grid_backward_binned_scratch_opts(64, nullptr, L, 2, 1, nullptr, &e, &c, &p) ==
                   DFHIP_EINVAL, "null offsets rejected");
        expect(dfhip_grid_encode_backward_binned_opts(4, DFHIP_F16, nullptr, nullptr, 1.0f, nullptr,
                                                      off.data(), nullptr, 0, nullptr, 3, 2, L,
                                                      0.5f, 16, 1, 0, 1, 0.0f, nullptr, nullptr,
                                                      nullptr, 0, nullptr, nullptr) == DFHIP_EINVAL,
               "phase 4 rejected");
        expect(dfhip_grid_encode_backward_binned_opts(3, DFHIP_F16, nullptr, nullptr, 1.0f, nullptr,
                                                      off.data(), nullptr, 0, nullptr, 3, 2, L,
                                                      0.5f, 16, 1, 0, 1, 0.0f, nullptr, nullptr,
                                                      nullptr, 0, nullptr, nullptr) == DFHIP_EINVAL,
               "null buffers rejected");
    }
    std::printf("gridbin host ASan driver: %d failure(s)\n", failures);
    return failures != 0;
}
