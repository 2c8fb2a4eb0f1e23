// Host-side sanitizer run of the C ABI (ASan/UBSan on the C-ABI shim). Built by
// tests/asan/build.sh (from tests/test_capi_sanitizers.py): the library sources with
// -fsanitize=address,undefined on the host pass only (no GPU needed). Every call below returns before
// any launch: argument validation, error codes and messages, and the size / layout arithmetic
// (workspace and packed-weight sizes, the image tile grid) over a sweep of shapes. Exits 0 when
// every expectation holds; the sanitizers abort on the first memory or UB error.
#include <stdio.h>
#include <string.h>

#include <vector>

#include "mcgmil.h"
#include "mcgmil_features.h"
#include "mcgmil_image.h"

static int failures = 0;
#define EXPECT(cond)                                                        \
    do {                                                                    \
        if (!(cond)) {                                                      \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            ++failures;                                                     \
        }                                                                   \
    } while (0)

static mcgmil_args base_args() {
    mcgmil_args a;
    memset(&a, 0, sizeof a);
    a.L = 512; a.D = 128; a.C = 2; a.G = 2; a.T = 100; a.num_bags = 1; a.total_rows = 2048;
    a.h_dtype = MCGMIL_BF16;
    a.bag_offsets = reinterpret_cast<const int32_t*>(0x1000);
    a.p_feat = a.p_att = 0.1f;
    return a;
}

static void expect_error(int rc, int code) {
    EXPECT(rc == code);
    const char* msg = mcgmil_last_error();
    EXPECT(msg != nullptr && strlen(msg) > 0);     // reads the thread-local message
}

static void mcdo_sizes() {
    // a sweep of head shapes and batch sizes through both size queries
    const int Ls[] = {32, 64, 96, 512, 1024, 2048};
    const int Ds[] = {16, 48, 128, 256};
    for (int L : Ls)
        for (int D : Ds)
            for (int C = 1; C <= 4; ++C)
                for (int G : {1, C}) {
                    mcgmil_args a = base_args();
                    a.L = L; a.D = D; a.C = C; a.G = G;
                    for (long long rows : {0LL, 1LL, 37LL, 2048LL, 1LL << 20}) {
                        a.total_rows = rows;
                        size_t ws = 0, pw = 0;
                        EXPECT(mcgmil_workspace_size(&a, &ws) == MCGMIL_OK);
                        EXPECT(mcgmil_packed_weights_size(&a, &pw) == MCGMIL_OK);
                        size_t want = (size_t)(2 * G * (D / 16) + 1) * (L / 32) * 512 * 2;
                        EXPECT(pw == want);
                        EXPECT(ws >= pw);
                    }
                }
}

static void mcdo_errors() {
    size_t n = 0;
    expect_error(mcgmil_workspace_size(nullptr, &n), MCGMIL_E_INVALID);
    mcgmil_args a = base_args();
    expect_error(mcgmil_workspace_size(&a, nullptr), MCGMIL_E_INVALID);
    a.L = 100;  expect_error(mcgmil_workspace_size(&a, &n), MCGMIL_E_UNSUPPORTED); a = base_args();
    a.L = 4096; expect_error(mcgmil_workspace_size(&a, &n), MCGMIL_E_UNSUPPORTED); a = base_args();
    a.D = 20;   expect_error(mcgmil_workspace_size(&a, &n), MCGMIL_E_UNSUPPORTED); a = base_args();
    a.C = 5;    expect_error(mcgmil_workspace_size(&a, &n), MCGMIL_E_UNSUPPORTED); a = base_args();
    a.G = 3;    expect_error(mcgmil_workspace_size(&a, &n), MCGMIL_E_INVALID); a = base_args();
    a.T = 0;    expect_error(mcgmil_workspace_size(&a, &n), MCGMIL_E_INVALID); a = base_args();
    a.num_bags = 0; expect_error(mcgmil_workspace_size(&a, &n), MCGMIL_E_INVALID); a = base_args();
    a.p_feat = 1.5f; expect_error(mcgmil_workspace_size(&a, &n), MCGMIL_E_INVALID); a = base_args();
    a.h_dtype = 7; expect_error(mcgmil_workspace_size(&a, &n), MCGMIL_E_INVALID); a = base_args();
    a.bag_offsets = nullptr; expect_error(mcgmil_workspace_size(&a, &n), MCGMIL_E_INVALID); a = base_args();
    a.uniform_bag_rows = 7; expect_error(mcgmil_workspace_size(&a, &n), MCGMIL_E_INVALID); a = base_args();
    a.total_rows = 1LL << 40; expect_error(mcgmil_workspace_size(&a, &n), MCGMIL_E_UNSUPPORTED);
    // forward: fails on the workspace / pointer checks before any launch
    a = base_args();
    expect_error(mcgmil_mcdo_forward(&a, nullptr), MCGMIL_E_WORKSPACE);
    std::vector<unsigned char> ws(1 << 20);
    a.workspace = ws.data() + 1;                     // misaligned (and too small)
    a.workspace_bytes = ws.size() - 1;
    EXPECT(mcgmil_mcdo_forward(&a, nullptr) != MCGMIL_OK);
    a = base_args();
    a.packed_w = reinterpret_cast<void*>(0x1000);
    a.total_rows = 0; a.T = 1;
    size_t need = 0;
    EXPECT(mcgmil_workspace_size(&a, &need) == MCGMIL_OK);
    std::vector<unsigned char> ws2(need + 512);
    a.workspace = reinterpret_cast<void*>(((uintptr_t)ws2.data() + 255) & ~(uintptr_t)255);
    a.workspace_bytes = need;
    expect_error(mcgmil_gate_scores(&a, nullptr), MCGMIL_E_INVALID);   // NULL bias vectors
    expect_error(mcgmil_softmax_pool(&a, nullptr), MCGMIL_E_INVALID);  // NULL Y
    uint8_t* none = nullptr;
    expect_error(mcgmil_feature_keep(&a, none, nullptr), MCGMIL_E_INVALID);
    expect_error(mcgmil_attention_keep(&a, none, nullptr), MCGMIL_E_INVALID);
    expect_error(mcgmil_pack_weights(&a, nullptr, nullptr), MCGMIL_E_INVALID);
    EXPECT(mcgmil_abi_version() == MCGMIL_ABI_VERSION);
    EXPECT(mcgmil_args_size() == sizeof(mcgmil_args));
}

static void image_grid() {
    // tile grids over a sweep of image / patch / overlap shapes (host arithmetic + vectors)
    for (int H : {1, 7, 224, 300, 7036})
        for (int W : {1, 5, 224, 2800})
            for (int ps : {1, 3, 64, 224})
                for (double ov : {0.0, 0.5, 0.75, 0.9}) {
                    mcgmil_image_args a;
                    memset(&a, 0, sizeof a);
                    a.height = H; a.width = W; a.channels = 3; a.patch_size = ps; a.overlap = ov;
                    a.empty_thresh = 0.5; a.bag_size = -1; a.image_dtype = MCGMIL_F32;
                    a.out_dtype = MCGMIL_F32; a.T = 4; a.C = 2; a.k = 1;
                    a.ld_row = W; a.ld_channel = (int64_t)H * W;
                    int32_t nt = -1, nr = -1, nc = -1;
                    const int rc = mcgmil_tile_grid(&a, nullptr, &nt, &nr, &nc);
                    if (ps > H || ps > W) {
                        EXPECT(rc != MCGMIL_OK);
                        continue;
                    }
                    if (rc != MCGMIL_OK) continue;     // a stride of 0 is rejected
                    EXPECT(nt == nr * nc && nt > 0);
                    std::vector<int64_t> tiles((size_t)nt * 6);
                    EXPECT(mcgmil_tile_grid(&a, tiles.data(), &nt, nullptr, nullptr) == MCGMIL_OK);
                    for (int i = 0; i < nt; ++i) {
                        EXPECT(tiles[6 * i] >= 0 && tiles[6 * i] + ps <= H);
                        EXPECT(tiles[6 * i + 1] >= 0 && tiles[6 * i + 1] + ps <= W);
                    }
                    size_t ws = 0;
                    EXPECT(mcgmil_image_workspace_size(&a, &ws) == MCGMIL_OK);
                }
    mcgmil_image_args a;
    memset(&a, 0, sizeof a);
    int32_t nt = 0;
    EXPECT(mcgmil_tile_grid(&a, nullptr, &nt, nullptr, nullptr) != MCGMIL_OK);
    EXPECT(mcgmil_tile_grid(nullptr, nullptr, &nt, nullptr, nullptr) != MCGMIL_OK);
    EXPECT(mcgmil_image_to_bag(&a, nullptr) != MCGMIL_OK);
    EXPECT(mcgmil_attention_maps(&a, nullptr) != MCGMIL_OK);
    EXPECT(mcgmil_image_args_size() == sizeof(mcgmil_image_args));
}

static void features_errors() {
    mcgmil_bn_args b;
    memset(&b, 0, sizeof b);
    size_t n = 0;
    EXPECT(mcgmil_bn_workspace_size(&b, &n) != MCGMIL_OK);     // channels 0
    EXPECT(mcgmil_bn_workspace_size(nullptr, &n) != MCGMIL_OK);
    b.rows = 1000; b.channels = 64; b.dtype = MCGMIL_BF16; b.eps = 1e-5;
    b.x = reinterpret_cast<const void*>(0x1000);                // never dereferenced on the host
    b.y = reinterpret_cast<void*>(0x2000);
    EXPECT(mcgmil_bn_workspace_size(&b, &n) == MCGMIL_OK);
    b.channels = 12;
    EXPECT(mcgmil_bn_workspace_size(&b, &n) == MCGMIL_E_UNSUPPORTED);
    b.channels = 64; b.pool_kernel = 3; b.pool_stride = 2; b.pool_pad = 1;   // N*H*W != rows
    EXPECT(mcgmil_bn_workspace_size(&b, &n) != MCGMIL_OK);
    b.pool_kernel = 0; b.x = nullptr;
    EXPECT(mcgmil_batchnorm_act(&b, nullptr) != MCGMIL_OK);     // NULL x
    EXPECT(mcgmil_bn_args_size() == sizeof(mcgmil_bn_args));
    mcgmil_conv_args c;
    memset(&c, 0, sizeof c);
    int32_t parts = -1, sup = -1;
    EXPECT(mcgmil_conv2d(&c, nullptr) != MCGMIL_OK);
    EXPECT(mcgmil_conv2d(nullptr, nullptr) != MCGMIL_OK);
    c.batch = 2; c.height = 56; c.width = 56; c.in_channels = 64; c.out_channels = 64;
    c.kernel_h = c.kernel_w = 3; c.stride = 1; c.pad = 1;
    EXPECT(mcgmil_conv_stats_parts(&c, &parts) == MCGMIL_OK && parts >= 0);
    EXPECT(mcgmil_conv_input_bn(&c, &sup) == MCGMIL_OK && (sup == 0 || sup == 1));
    EXPECT(mcgmil_conv2d(&c, nullptr) != MCGMIL_OK);            // NULL tensors
    EXPECT(mcgmil_conv_args_size() == sizeof(mcgmil_conv_args));
    mcgmil_stem_args s;
    memset(&s, 0, sizeof s);
    EXPECT(mcgmil_stem_packed_size(&s, &n) != MCGMIL_OK);
    EXPECT(mcgmil_stem_workspace_size(nullptr, &n) != MCGMIL_OK);
    EXPECT(mcgmil_stem_forward(&s, nullptr) != MCGMIL_OK);
    EXPECT(mcgmil_stem_args_size() == sizeof(mcgmil_stem_args));
}

int main() {
    mcdo_sizes();
    mcdo_errors();
    image_grid();
    features_errors();
    printf("capi_host_check: %d failure(s)\n", failures);
    return failures ? 1 : 0;
}
