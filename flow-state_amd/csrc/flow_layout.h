// Raw (state_dict order) and packed (MFMA-fragment) parameter layouts of one
// circular-RQS coupling layer.  Shared by the host C-ABI and the device code.
#pragma once
#include <stdint.h>
#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#endif

#ifdef __HIPCC__
#define FS_HD __host__ __device__ __forceinline__
#else
#define FS_HD inline
#endif

namespace fs {

constexpr int kRows = 64;     // chains per workgroup (= lanes of a wave: lane-per-chain spline)
constexpr int kWaves = 8;     // waves per workgroup (2 per SIMD: one wave's VALU hides under the other's MFMAs)
constexpr int kThreads = kRows * kWaves;
constexpr int kMaxN = 64;     // particles (energy kernel: lane-per-particle, nbr mask in one u64)
constexpr int kMaxK = 32;     // spline bins (one 32-column MFMA tile per parameter group)

FS_HD int64_t rup(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

struct RawLayout {  // offsets in floats within one layer of the raw buffer
    int64_t win, bin, blocks, block_stride, wf, bf, uw, uh, ud, stride;
    // within a block
    static constexpr int64_t bn0 = 0;  // + H*{0: weight, 1: bias, 2: mean, 3: var}
    FS_HD static int64_t w0(int64_t H) { return 4 * H; }
    FS_HD static int64_t b0(int64_t H) { return 4 * H + H * H; }
    FS_HD static int64_t bn1(int64_t H) { return 5 * H + H * H; }
    FS_HD static int64_t w1(int64_t H) { return 9 * H + H * H; }
    FS_HD static int64_t b1(int64_t H) { return 9 * H + 2 * H * H; }
};

FS_HD RawLayout raw_layout(int N, int H, int nb, int K) {
    RawLayout r;
    const int64_t D = 2 * N, P = 3 * K + 1;
    r.win = 0;
    r.bin = H * D;
    r.blocks = r.bin + H;
    r.block_stride = 2 * (int64_t)H * H + 10 * (int64_t)H;
    r.wf = r.blocks + nb * r.block_stride;
    r.bf = r.wf + N * P * H;
    r.uw = r.bf + N * P;
    r.uh = r.uw + (int64_t)N * K;
    r.ud = r.uh + (int64_t)N * K;
    r.stride = r.ud + (int64_t)N * (K + 1);
    return r;
}

// Packed layout of one layer (offsets in floats, every section 64-float aligned).
// GEMM B operands are stored as [tile][k-group][lane][4]: tile = 32 output
// columns, k-group = 8 reduction indices; lane l (h = l>>5, c = l&31) holds
// W[col = 32*tile + c][k = 8*g + 4*h + j] for j = 0..3 -> one 16-byte load per
// lane feeds four v_mfma_f32_32x32x2_f32 steps (k = 8g+j and 8g+4+j).
// The derivative rows of the final layer (d_0..d_K of every transform feature,
// coupling.py:327-342) are NOT a GEMM operand: a chain's spline reads only d_bin and
// d_bin+1 (splines.py:157-158), so the f32 kernel gathers those two rows per lane and
// takes their dot products with the chain's hidden vector.  They are stored
// [feature][quad q = k/4][row 0..K][4] (`wd`): for one quad the 64 lanes of a wave
// read 16-byte pieces of one (K+1)*16-byte stretch, offset by their bins.
struct PackLayout {
    int kg_in;       // k-groups of the initial layer (ceil(2N/8))
    int kg_h;        // k-groups of an H-input layer (H/8)
    int ntt;         // ceil(N/32) (v_bt: the split image's d_K biases)
    int64_t win;     // [H/32][kg_in][64][4]
    int64_t blocks;  // nb x { W0 [H/32][kg_h][64][4], W1 [...] }
    int64_t block_stride;
    int64_t wf;      // final layer, per feature j: 2 tiles (widths, heights)
    int64_t wd;      // final layer derivative rows, per feature j: [H/4][K+1][4]
    int64_t vec;     // s_h[H]; nb x {a0,c0',a1,c1'}[H]; bf[N][3][32]; bt[ntt*32]; bd[N][K+1] (pack_vec_kernel)
    int64_t v_blocks, v_bf, v_bt, v_bd;
    int64_t unc;     // unconditional knots: [N][3][K+1] = cumwidths, cumheights, derivatives
    int64_t stride;
};

FS_HD PackLayout pack_layout(int N, int H, int nb, int K) {
    PackLayout p;
    p.kg_in = (int)((2 * N + 7) / 8);
    p.kg_h = H / 8;
    p.ntt = (N + 31) / 32;
    const int64_t tiles_h = H / 32;
    p.win = 0;
    p.blocks = rup(p.win + tiles_h * p.kg_in * 256, 64);
    p.block_stride = 2 * tiles_h * p.kg_h * 256;
    p.wf = rup(p.blocks + nb * p.block_stride, 64);
    p.wd = rup(p.wf + (int64_t)N * 2 * p.kg_h * 256, 64);
    p.vec = rup(p.wd + (int64_t)N * H * (K + 1), 64);
    p.v_blocks = H;
    p.v_bf = p.v_blocks + 4 * (int64_t)H * nb;
    p.v_bt = p.v_bf + (int64_t)N * 96;
    p.v_bd = p.v_bt + p.ntt * 32;
    p.unc = rup(p.vec + p.v_bd + (int64_t)N * (K + 1), 64);
    p.stride = rup(p.unc + (int64_t)N * 3 * (K + 1), 64);
    return p;
}

// X (activation tile) row width in floats: max(H, 2*kMaxN) so that it holds the
// H hidden units and the 2N <= 128 periodic input features.  Rows are padded by 4 floats (one 16-byte
// slot): ds_read_b128 A fragments (16 rows x one slot per lane group) and the
// epilogue's ds_write_b32 (32 consecutive columns of one row) are conflict-free,
// and every address is base + immediate offset.
FS_HD int flow_xw(int H) { return H < 2 * kMaxN ? 2 * kMaxN : H; }

struct LdsLayout {
    int x, coord, ld, total;  // byte offsets
    int xw, xs, cstride;
};

FS_HD LdsLayout lds_layout(int N, int H) {
    LdsLayout l;
    l.xw = flow_xw(H);
    l.xs = l.xw + 4;
    l.cstride = 2 * N + 1;                 // odd stride: lane-per-row reads are conflict-free
    l.x = 0;
    l.coord = l.x + kRows * l.xs * 4;
    l.ld = (int)rup(l.coord + kRows * l.cstride * 4, 16);
    l.total = l.ld + kWaves * kRows * 4 + 16;
    return l;
}

// ---------------------------------------------------------------------------
// Split-bf16 image (fs_flow_dims.precision = 1: P = 3 planes, 6 products;
// precision = 2: P = 2 planes, 3 products).  Every f32 weight w is stored as P
// bf16 planes w = w_0 + w_1 (+ w_2), each the round-to-nearest-even bf16 of the
// remainder of the previous ones.  GEMM A operands of v_mfma_f32_32x32x16_bf16
// (the conditioner runs transposed: C^T = W . X^T, so the weights are the A
// operand and the accumulator lane is the chain) are 1 KiB fragments
// [tile (32 output rows)][k-step (16 inputs)][plane][lane][8 bf16]: lane l
// (r = l & 31, h = l >> 5) holds W[32 tile + r][16 s + 8 h + j], j = 0..7.
// Offsets are in floats (1 fragment = 256 floats).  The vector section (folded
// BatchNorm, biases) and the unconditional knots are those of PackLayout, at
// the same distance from each other (pack_vec_kernel writes both images).
// ---------------------------------------------------------------------------
FS_HD int split_planes(int precision) { return precision == 1 ? 3 : 2; }

struct SplitLayout {
    int P;            // planes
    int kst_in;       // k-steps of the initial layer (ceil(2N/16))
    int kst_h;        // k-steps of an H-input layer (H/16)
    int nfw;          // transform features per wave (ceil(N/8)); wave w owns [w nfw, (w+1) nfw)
    int64_t win;      // [H/32][kst_in][P] fragments
    int64_t blocks;   // nb x { W0 [H/32][kst_h][P], W1 [...] }
    int64_t block_stride;
    int64_t wf;       // final layer: per feature j, 3 tiles (widths, heights, d_0..d_{K-1})
    int64_t wt;       // per wave: one tile whose rows r < nfw are d_K of feature w nfw + r
    int64_t vec;      // PackLayout's vector section
    int64_t unc;      // PackLayout's unconditional knots
    int64_t stride;
};

FS_HD SplitLayout split_layout(int N, int H, int nb, int K, int precision) {
    SplitLayout s;
    const PackLayout p = pack_layout(N, H, nb, K);
    s.P = split_planes(precision);
    s.kst_in = (2 * N + 15) / 16;
    s.kst_h = H / 16;
    s.nfw = (N + 7) / 8;
    const int64_t frag = 256 * (int64_t)s.P;  // floats per (tile, k-step), all planes
    const int64_t tiles_h = H / 32;
    s.win = 0;
    s.blocks = s.win + tiles_h * s.kst_in * frag;
    s.block_stride = 2 * tiles_h * s.kst_h * frag;
    s.wf = s.blocks + nb * s.block_stride;
    s.wt = s.wf + (int64_t)N * 3 * s.kst_h * frag;
    s.vec = s.wt + (int64_t)8 * s.kst_h * frag;
    s.unc = s.vec + (p.unc - p.vec);
    s.stride = rup(s.unc + (int64_t)N * 3 * (K + 1), 64);
    return s;
}

// LDS of the split kernel: activations [64 chains][P planes][xw + 8] bf16 (a
// chain's planes are adjacent, so every fragment address of a GEMM is one base
// VGPR + a 16-bit immediate; the 16-byte pad per plane row keeps the 32 rows of
// a ds_read_b128 fragment and the ds_write_b64 epilogue stores conflict-free),
// then coordinates, tail values, log-det partials.  `plane` = bytes between the
// planes of one chain, `xsb` = bytes between chains.
struct SplitLds {
    int xw, xsb, plane, coord, tail, ld, total, cstride, tstride;
};

FS_HD SplitLds split_lds(int N, int H, int P) {
    SplitLds l;
    const int in16 = (2 * N + 15) / 16 * 16;
    l.xw = H > in16 ? H : in16;
    l.plane = 2 * l.xw + 16;
    l.xsb = P * l.plane;
    l.cstride = 2 * N + 1;
    l.tstride = 8 * ((N + 7) / 8) + 1;
    l.coord = kRows * l.xsb;
    l.tail = (int)rup(l.coord + kRows * l.cstride * 4, 16);
    l.ld = (int)rup(l.tail + kRows * l.tstride * 4, 16);
    l.total = l.ld + kWaves * kRows * 4 + 16;
    return l;
}

}  // namespace fs
