// jpeg.cpp -- the JPEG half of the densify CLI's image ingest.
//
// The reference loads every view with cv::imread(filename) (modules/core/
// types.cpp:7-11, called from PMVS::AddCamera, methods/pmvs/pmvs.cpp:11-20):
// IMREAD_COLOR, i.e. BGR8, decoded by libjpeg(-turbo) with its defaults --
// the accurate integer IDCT (JDCT_ISLOW, jidctint.c), "fancy" triangle-filter
// chroma upsampling (jdsample.c), the fixed-point YCbCr->RGB tables of
// jdcolor.c -- and then EXIF orientation applied (imread without
// IMREAD_IGNORE_ORIENTATION).  This file restates that decode for the formats
// scene folders hold: baseline and extended sequential Huffman (SOF0/SOF1) and
// progressive Huffman (SOF2), 8-bit, one (gray) or three (YCbCr or Adobe RGB)
// components, any integer sampling factors, restart intervals.  Arithmetic
// coding, 12-bit samples, CMYK/YCCK and lossless JPEG are rejected with a
// message (cv::imread reads some of them; scene folders do not hold them).
//
// Pinned by tests/golden/jpeg_*.npz: files written by Pillow's libjpeg-turbo
// encoder and the BGR arrays its decoder returns (tests/golden/make_golden_jpeg.py).
#include "scene_io.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <vector>

namespace dpio {
namespace {

// zigzag index -> natural (row-major) coefficient index
const int kNatural[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                          12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                          35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                          58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct JpegError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// ---- Huffman tables (canonical codes, JPEG Annex C) ---------------------------
struct Huffman {
    bool present = false;
    uint8_t vals[256] = {};
    int mincode[17] = {}, maxcode[18] = {}, valoff[17] = {};
    uint16_t look[512] = {}; // 9-bit lookahead: (length << 8) | value, 0 = longer code
    int max_sym = 0;         // largest symbol (a DC table's must be <= 15)

    void build(const uint8_t counts[16], const uint8_t *v, int nv)
    {
        std::memcpy(vals, v, (size_t)nv);
        std::memset(look, 0, sizeof(look));
        max_sym = 0;
        for (int i = 0; i < nv; ++i)
            max_sym = std::max(max_sym, (int)v[i]);
        int code = 0, k = 0;
        for (int l = 1; l <= 16; ++l) {
            valoff[l] = k;
            mincode[l] = code;
            for (int i = 0; i < counts[l - 1]; ++i, ++k, ++code) {
                if (l <= 9)
                    for (int f = 0; f < (1 << (9 - l)); ++f)
                        look[(code << (9 - l)) | f] = (uint16_t)(l << 8 | vals[k]);
            }
            maxcode[l] = counts[l - 1] ? code - 1 : -1;
            if (code > (1 << l))
                throw JpegError("bad Huffman table");
            code <<= 1;
        }
        maxcode[17] = 0x7fffffff;
        present = true;
    }
};

// ---- entropy-coded segment reader --------------------------------------------
// Like libjpeg's jdhuff.c fill_bit_buffer: on reaching a marker it stops
// consuming bytes and feeds zero bits (a valid stream never reads them).
struct BitReader {
    const uint8_t *p;
    size_t n, pos;
    uint64_t acc = 0;
    int cnt = 0;
    bool at_marker = false;

    void fill()
    {
        while (cnt <= 56) {
            unsigned b = 0;
            if (!at_marker && pos < n) {
                b = p[pos];
                if (b == 0xFF) {
                    unsigned b2 = pos + 1 < n ? p[pos + 1] : 0xD9;
                    if (b2 == 0x00) {
                        pos += 2;
                    } else {
                        at_marker = true;
                        b = 0;
                    }
                } else {
                    ++pos;
                }
            }
            acc |= (uint64_t)b << (56 - cnt);
            cnt += 8;
        }
    }
    int bits(int k)
    {
        if (k == 0)
            return 0;
        fill();
        const int v = (int)(acc >> (64 - k));
        acc <<= k;
        cnt -= k;
        return v;
    }
    int bit() { return bits(1); }
    int decode(const Huffman &h)
    {
        if (!h.present)
            throw JpegError("scan uses an undefined Huffman table");
        fill();
        const uint16_t e = h.look[acc >> 55];
        if (e) {
            acc <<= e >> 8;
            cnt -= e >> 8;
            return e & 0xff;
        }
        for (int l = 10; l <= 16; ++l) {
            const int code = (int)(acc >> (64 - l));
            if (code <= h.maxcode[l]) {
                acc <<= l;
                cnt -= l;
                return h.vals[h.valoff[l] + code - h.mincode[l]];
            }
        }
        throw JpegError("corrupt Huffman code");
    }
    // RSTn: drop the buffered bits, skip fill bytes and the marker
    void restart()
    {
        acc = 0;
        cnt = 0;
        at_marker = false;
        while (pos + 1 < n && !(p[pos] == 0xFF && p[pos + 1] >= 0xD0 && p[pos + 1] <= 0xD7))
            ++pos;
        if (pos + 1 >= n)
            throw JpegError("missing restart marker");
        pos += 2;
    }
};

inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

// ---- components ------------------------------------------------------------
struct Component {
    int id = 0, h = 1, v = 1, tq = 0;
    int td = 0, ta = 0;     // Huffman table selectors of the current scan
    int bw = 0, bh = 0;     // coefficient blocks allocated (MCU-padded)
    int dw = 0, dh = 0;     // downsampled_width / _height (libjpeg)
    int pred = 0;           // DC predictor
    std::vector<int16_t> coef; // bw*bh blocks x 64, natural order
    std::vector<uint8_t> plane; // IDCT output, stride 8*bw
};

// jidctint.c jpeg_idct_islow: 13-bit constants, PASS1_BITS 2, the post-IDCT
// range-limit table indexed by (x & 1023) (jdmaster.c prepare_range_limit_table)
const long kC0298 = 2446, kC0390 = 3196, kC0541 = 4433, kC0765 = 6270, kC0899 = 7373, kC1175 = 9633,
           kC1501 = 12299, kC1847 = 15137, kC1961 = 16069, kC2053 = 16819, kC2562 = 20995, kC3072 = 25172;

struct IdctRange {
    uint8_t t[1024];
    IdctRange()
    {
        for (int i = 0; i < 1024; ++i)
            t[i] = i < 128 ? (uint8_t)(128 + i) : i < 512 ? 255 : i < 896 ? 0 : (uint8_t)(i - 896);
    }
};
const IdctRange kRange;

inline long descale(long x, int n) { return (x + (1L << (n - 1))) >> n; }

void idct_islow(const int16_t *in, const uint16_t *q, uint8_t *out, int stride)
{
    int ws[64];
    for (int c = 0; c < 8; ++c) {
        const int16_t *ip = in + c;
        const uint16_t *qp = q + c;
        long z2 = (long)ip[16] * qp[16], z3 = (long)ip[48] * qp[48];
        long z1 = (z2 + z3) * kC0541;
        const long t2 = z1 + z3 * -kC1847, t3 = z1 + z2 * kC0765;
        z2 = (long)ip[0] * qp[0];
        z3 = (long)ip[32] * qp[32];
        const long t0 = (z2 + z3) << 13, t1 = (z2 - z3) << 13;
        const long t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
        long o0 = (long)ip[56] * qp[56], o1 = (long)ip[40] * qp[40], o2 = (long)ip[24] * qp[24],
             o3 = (long)ip[8] * qp[8];
        z1 = o0 + o3;
        z2 = o1 + o2;
        z3 = o0 + o2;
        long z4 = o1 + o3;
        const long z5 = (z3 + z4) * kC1175;
        o0 *= kC0298;
        o1 *= kC2053;
        o2 *= kC3072;
        o3 *= kC1501;
        z1 *= -kC0899;
        z2 *= -kC2562;
        z3 = z3 * -kC1961 + z5;
        z4 = z4 * -kC0390 + z5;
        o0 += z1 + z3;
        o1 += z2 + z4;
        o2 += z2 + z3;
        o3 += z1 + z4;
        ws[c + 0] = (int)descale(t10 + o3, 11);
        ws[c + 56] = (int)descale(t10 - o3, 11);
        ws[c + 8] = (int)descale(t11 + o2, 11);
        ws[c + 48] = (int)descale(t11 - o2, 11);
        ws[c + 16] = (int)descale(t12 + o1, 11);
        ws[c + 40] = (int)descale(t12 - o1, 11);
        ws[c + 24] = (int)descale(t13 + o0, 11);
        ws[c + 32] = (int)descale(t13 - o0, 11);
    }
    for (int r = 0; r < 8; ++r) {
        const int *w = ws + 8 * r;
        uint8_t *op = out + (size_t)r * stride;
        long z2 = w[2], z3 = w[6];
        long z1 = (z2 + z3) * kC0541;
        const long t2 = z1 + z3 * -kC1847, t3 = z1 + z2 * kC0765;
        const long t0 = ((long)w[0] + w[4]) << 13, t1 = ((long)w[0] - w[4]) << 13;
        const long t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
        long o0 = w[7], o1 = w[5], o2 = w[3], o3 = w[1];
        z1 = o0 + o3;
        z2 = o1 + o2;
        z3 = o0 + o2;
        long z4 = o1 + o3;
        const long z5 = (z3 + z4) * kC1175;
        o0 *= kC0298;
        o1 *= kC2053;
        o2 *= kC3072;
        o3 *= kC1501;
        z1 *= -kC0899;
        z2 *= -kC2562;
        z3 = z3 * -kC1961 + z5;
        z4 = z4 * -kC0390 + z5;
        o0 += z1 + z3;
        o1 += z2 + z4;
        o2 += z2 + z3;
        o3 += z1 + z4;
        op[0] = kRange.t[descale(t10 + o3, 18) & 1023];
        op[7] = kRange.t[descale(t10 - o3, 18) & 1023];
        op[1] = kRange.t[descale(t11 + o2, 18) & 1023];
        op[6] = kRange.t[descale(t11 - o2, 18) & 1023];
        op[2] = kRange.t[descale(t12 + o1, 18) & 1023];
        op[5] = kRange.t[descale(t12 - o1, 18) & 1023];
        op[3] = kRange.t[descale(t13 + o0, 18) & 1023];
        op[4] = kRange.t[descale(t13 - o0, 18) & 1023];
    }
}

inline uint8_t clamp255(int x) { return (uint8_t)(x < 0 ? 0 : x > 255 ? 255 : x); }

// jdsample.c: one component's IDCT plane -> width x height full-resolution
// samples.  Fancy (triangle) filters for 2h1v, 1h2v and 2h2v, edge rows and
// columns replicated as jdmainct.c's context pointers do; plain replication
// for every other integer ratio.
std::vector<uint8_t> upsample(const Component &c, int hmax, int vmax, int width, int height)
{
    const int hx = hmax / c.h, vx = vmax / c.v, stride = 8 * c.bw;
    const int dw = c.dw, dh = c.dh;
    const uint8_t *in = c.plane.data();
    std::vector<uint8_t> out((size_t)width * height);
    auto row = [&](int r) { return in + (size_t)(r < 0 ? 0 : r >= dh ? dh - 1 : r) * stride; };
    const int ow = hx * dw; // output row before cropping to width
    std::vector<uint8_t> tmp((size_t)ow);
    for (int y = 0; y < height; ++y) {
        const int r = y / vx;
        const uint8_t *src = row(r);
        if (hx == 1 && vx == 1) {
            std::memcpy(&out[(size_t)y * width], src, (size_t)width);
            continue;
        }
        if (hx == 2 && vx == 2 && dw > 2) { // h2v2_fancy_upsample
            const uint8_t *nb = (y & 1) ? row(r + 1) : row(r - 1);
            int thiscol = src[0] * 3 + nb[0], nextcol = src[1] * 3 + nb[1], lastcol;
            uint8_t *o = tmp.data();
            *o++ = (uint8_t)((thiscol * 4 + 8) >> 4);
            *o++ = (uint8_t)((thiscol * 3 + nextcol + 7) >> 4);
            lastcol = thiscol;
            thiscol = nextcol;
            for (int x = 2; x < dw; ++x) {
                nextcol = src[x] * 3 + nb[x];
                *o++ = (uint8_t)((thiscol * 3 + lastcol + 8) >> 4);
                *o++ = (uint8_t)((thiscol * 3 + nextcol + 7) >> 4);
                lastcol = thiscol;
                thiscol = nextcol;
            }
            *o++ = (uint8_t)((thiscol * 3 + lastcol + 8) >> 4);
            *o++ = (uint8_t)((thiscol * 4 + 7) >> 4);
        } else if (hx == 2 && vx == 1 && dw > 2) { // h2v1_fancy_upsample
            uint8_t *o = tmp.data();
            int inv = src[0];
            *o++ = (uint8_t)inv;
            *o++ = (uint8_t)((inv * 3 + src[1] + 2) >> 2);
            for (int x = 1; x < dw - 1; ++x) {
                inv = src[x] * 3;
                *o++ = (uint8_t)((inv + src[x - 1] + 1) >> 2);
                *o++ = (uint8_t)((inv + src[x + 1] + 2) >> 2);
            }
            inv = src[dw - 1];
            *o++ = (uint8_t)((inv * 3 + src[dw - 2] + 1) >> 2);
            *o++ = (uint8_t)inv;
        } else if (hx == 1 && vx == 2) { // h1v2_fancy_upsample
            const uint8_t *nb = (y & 1) ? row(r + 1) : row(r - 1);
            const int bias = (y & 1) ? 2 : 1;
            for (int x = 0; x < dw; ++x)
                tmp[x] = (uint8_t)((src[x] * 3 + nb[x] + bias) >> 2);
        } else { // int_upsample / h2v1_upsample / h2v2_upsample: replication
            for (int x = 0; x < ow; ++x)
                tmp[x] = src[x / hx];
        }
        std::memcpy(&out[(size_t)y * width], tmp.data(), (size_t)width);
    }
    return out;
}

// EXIF orientation (APP1 "Exif\0\0", IFD0 tag 0x0112), 1 when absent
int exif_orientation(const uint8_t *a, size_t len)
{
    if (len < 14 || std::memcmp(a, "Exif\0\0", 6) != 0)
        return 1;
    const uint8_t *t = a + 6;
    const size_t tl = len - 6;
    bool le;
    if (t[0] == 'I' && t[1] == 'I')
        le = true;
    else if (t[0] == 'M' && t[1] == 'M')
        le = false;
    else
        return 1;
    auto u16 = [&](size_t o) -> unsigned { return le ? t[o] | t[o + 1] << 8 : t[o] << 8 | t[o + 1]; };
    auto u32 = [&](size_t o) -> size_t {
        return le ? (size_t)t[o] | (size_t)t[o + 1] << 8 | (size_t)t[o + 2] << 16 | (size_t)t[o + 3] << 24
                  : (size_t)t[o] << 24 | (size_t)t[o + 1] << 16 | (size_t)t[o + 2] << 8 | (size_t)t[o + 3];
    };
    const size_t ifd = u32(4);
    if (ifd + 2 > tl)
        return 1;
    const unsigned ne = u16(ifd);
    for (unsigned i = 0; i < ne; ++i) {
        const size_t e = ifd + 2 + 12 * (size_t)i;
        if (e + 12 > tl)
            break;
        if (u16(e) == 0x0112 && u16(e + 2) == 3) {
            const unsigned o = u16(e + 8);
            return o >= 1 && o <= 8 ? (int)o : 1;
        }
    }
    return 1;
}

// cv::imread's ApplyExifOrientation: flips / transposes of the BGR image
Image orient(const Image &im, int o)
{
    if (o == 1)
        return im;
    const bool tr = o >= 5;
    const int W = im.width, H = im.height;
    const int ow = tr ? H : W, oh = tr ? W : H;
    // after the optional transpose: flip horizontally (2, 6), both (3, 7), vertically (4, 8)
    const bool fx = o == 2 || o == 3 || o == 6 || o == 7, fy = o == 3 || o == 4 || o == 7 || o == 8;
    Image r;
    r.width = ow;
    r.height = oh;
    r.bgr.resize((size_t)ow * oh * 3);
    for (int y = 0; y < oh; ++y)
        for (int x = 0; x < ow; ++x) {
            const int ty = fy ? oh - 1 - y : y, tx = fx ? ow - 1 - x : x; // position before the flip
            const int sy = tr ? tx : ty, sx = tr ? ty : tx;
            std::memcpy(&r.bgr[((size_t)y * ow + x) * 3], &im.bgr[((size_t)sy * W + sx) * 3], 3);
        }
    return r;
}

class Decoder {
public:
    Decoder(const uint8_t *d, size_t n) : d_(d), n_(n) {}

    Image run()
    {
        if (n_ < 4 || d_[0] != 0xFF || d_[1] != 0xD8)
            throw JpegError("not a JPEG (no SOI)");
        size_t pos = 2;
        for (;;) {
            // next marker (fill bytes allowed)
            if (pos >= n_)
                throw JpegError("truncated (no EOI)");
            if (d_[pos] != 0xFF)
                throw JpegError("expected a marker");
            while (pos < n_ && d_[pos] == 0xFF)
                ++pos;
            if (pos >= n_)
                throw JpegError("truncated marker");
            const int m = d_[pos++];
            if (m == 0xD9)
                break; // EOI
            if (m >= 0xD0 && m <= 0xD7)
                continue; // stray RSTn
            if (pos + 2 > n_)
                throw JpegError("truncated segment");
            const size_t len = (size_t)d_[pos] << 8 | d_[pos + 1];
            if (len < 2 || pos + len > n_)
                throw JpegError("bad segment length");
            const uint8_t *s = d_ + pos + 2;
            const size_t sl = len - 2;
            pos += len;
            switch (m) {
            case 0xC0: case 0xC1: case 0xC2: frame(s, sl, m == 0xC2); break;
            case 0xC4: dht(s, sl); break;
            case 0xDB: dqt(s, sl); break;
            case 0xDD:
                if (sl < 2)
                    throw JpegError("bad DRI");
                restart_ = s[0] << 8 | s[1];
                break;
            case 0xDA: pos = scan(s, sl, pos); break;
            case 0xE0:
                if (sl >= 5 && std::memcmp(s, "JFIF\0", 5) == 0)
                    jfif_ = true;
                break;
            case 0xE1:
                if (orientation_ == 0)
                    orientation_ = exif_orientation(s, sl);
                break;
            case 0xEE:
                if (sl >= 12 && std::memcmp(s, "Adobe", 5) == 0) {
                    adobe_ = true;
                    adobe_transform_ = s[11];
                }
                break;
            case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9: case 0xCA: case 0xCB:
            case 0xCD: case 0xCE: case 0xCF:
                throw JpegError("unsupported JPEG process (lossless, hierarchical or arithmetic coding)");
            default: break; // APPn, COM, ...
            }
        }
        if (comps_.empty() || !any_scan_)
            throw JpegError("no image data");
        return orient(finish(), orientation_ ? orientation_ : 1);
    }

private:
    const uint8_t *d_;
    size_t n_;
    uint16_t q_[4][64] = {};
    Huffman dc_[4], ac_[4];
    std::vector<Component> comps_;
    int width_ = 0, height_ = 0, hmax_ = 1, vmax_ = 1, mcux_ = 0, mcuy_ = 0;
    int restart_ = 0, orientation_ = 0, adobe_transform_ = -1;
    bool progressive_ = false, jfif_ = false, adobe_ = false, any_scan_ = false;
    int eobrun_ = 0;

    void dqt(const uint8_t *s, size_t sl)
    {
        size_t i = 0;
        while (i < sl) {
            const int pq = s[i] >> 4, tq = s[i] & 15;
            if (tq > 3 || pq > 1 || i + 1 + 64 * (pq + 1) > sl)
                throw JpegError("bad DQT");
            for (int k = 0; k < 64; ++k)
                q_[tq][kNatural[k]] = pq ? (uint16_t)(s[i + 1 + 2 * k] << 8 | s[i + 2 + 2 * k]) : s[i + 1 + k];
            i += 1 + 64 * (pq + 1);
        }
    }

    void dht(const uint8_t *s, size_t sl)
    {
        size_t i = 0;
        while (i < sl) {
            if (i + 17 > sl)
                throw JpegError("bad DHT");
            const int tc = s[i] >> 4, th = s[i] & 15;
            int nv = 0;
            for (int l = 0; l < 16; ++l)
                nv += s[i + 1 + l];
            if (tc > 1 || th > 3 || nv > 256 || i + 17 + nv > sl)
                throw JpegError("bad DHT");
            (tc ? ac_ : dc_)[th].build(s + i + 1, s + i + 17, nv);
            i += 17 + nv;
        }
    }

    void frame(const uint8_t *s, size_t sl, bool prog)
    {
        if (!comps_.empty())
            throw JpegError("more than one frame");
        if (sl < 6 || s[0] != 8)
            throw JpegError("unsupported JPEG (need 8-bit samples)");
        progressive_ = prog;
        height_ = s[1] << 8 | s[2];
        width_ = s[3] << 8 | s[4];
        const int nc = s[5];
        if (width_ <= 0 || height_ <= 0)
            throw JpegError("unsupported JPEG (zero dimension / DNL)");
        if ((nc != 1 && nc != 3) || sl < 6 + 3 * (size_t)nc)
            throw JpegError("unsupported JPEG (need 1 or 3 components)");
        for (int c = 0; c < nc; ++c) {
            Component k;
            k.id = s[6 + 3 * c];
            k.h = s[7 + 3 * c] >> 4;
            k.v = s[7 + 3 * c] & 15;
            k.tq = s[8 + 3 * c];
            if (k.h < 1 || k.h > 4 || k.v < 1 || k.v > 4 || k.tq > 3)
                throw JpegError("bad component parameters");
            comps_.push_back(k);
            hmax_ = std::max(hmax_, k.h);
            vmax_ = std::max(vmax_, k.v);
        }
        mcux_ = (width_ + 8 * hmax_ - 1) / (8 * hmax_);
        mcuy_ = (height_ + 8 * vmax_ - 1) / (8 * vmax_);
        for (Component &k : comps_) {
            if (hmax_ % k.h || vmax_ % k.v)
                throw JpegError("unsupported (non-integer) sampling ratio");
            k.bw = mcux_ * k.h;
            k.bh = mcuy_ * k.v;
            k.dw = (int)(((long)width_ * k.h + hmax_ - 1) / hmax_);
            k.dh = (int)(((long)height_ * k.v + vmax_ - 1) / vmax_);
            k.coef.assign((size_t)k.bw * k.bh * 64, 0);
        }
    }

    // one block of a scan (jdhuff.c decode_mcu / jdphuff.c decode_mcu_*)
    void block(BitReader &br, Component &c, int16_t *b, int ss, int se, int ah, int al)
    {
        if (!progressive_) {
            const int t = br.decode(dc_[c.td]);
            c.pred += t ? extend(br.bits(t), t) : 0;
            b[0] = (int16_t)c.pred;
            for (int k = 1; k < 64; ++k) {
                const int rs = br.decode(ac_[c.ta]), r = rs >> 4, s = rs & 15;
                if (s) {
                    k += r;
                    if (k > 63)
                        throw JpegError("corrupt AC run");
                    b[kNatural[k]] = (int16_t)extend(br.bits(s), s);
                } else {
                    if (r != 15)
                        break;
                    k += 15;
                }
            }
            return;
        }
        if (ss == 0) { // DC scans
            if (ah == 0) {
                const int t = br.decode(dc_[c.td]);
                c.pred += t ? extend(br.bits(t), t) : 0;
                b[0] = (int16_t)(c.pred * (1 << al));
            } else if (br.bit()) {
                b[0] = (int16_t)(b[0] | (1 << al));
            }
            return;
        }
        if (ah == 0) { // AC first
            if (eobrun_ > 0) {
                --eobrun_;
                return;
            }
            for (int k = ss; k <= se; ++k) {
                const int rs = br.decode(ac_[c.ta]), r = rs >> 4, s = rs & 15;
                if (s) {
                    k += r;
                    if (k > 63)
                        throw JpegError("corrupt AC run");
                    b[kNatural[k]] = (int16_t)(extend(br.bits(s), s) * (1 << al));
                } else if (r == 15) {
                    k += 15;
                } else {
                    eobrun_ = 1 << r;
                    if (r)
                        eobrun_ += br.bits(r);
                    --eobrun_;
                    break;
                }
            }
            return;
        }
        // AC refinement (jdphuff.c decode_mcu_AC_refine)
        const int p1 = 1 << al, m1 = -1 * (1 << al);
        auto correct = [&](int16_t &v) {
            if (br.bit() && (v & p1) == 0)
                v = (int16_t)(v >= 0 ? v + p1 : v + m1);
        };
        int k = ss;
        if (eobrun_ == 0) {
            for (; k <= se; ++k) {
                const int rs = br.decode(ac_[c.ta]);
                int r = rs >> 4, s = rs & 15;
                if (s) {
                    s = br.bit() ? p1 : m1;
                } else if (r != 15) {
                    eobrun_ = 1 << r;
                    if (r)
                        eobrun_ += br.bits(r);
                    break;
                }
                do {
                    int16_t &v = b[kNatural[k]];
                    if (v != 0)
                        correct(v);
                    else if (--r < 0)
                        break;
                    ++k;
                } while (k <= se);
                if (s) {
                    if (k > 63)
                        throw JpegError("corrupt AC refinement");
                    b[kNatural[k]] = (int16_t)s;
                }
            }
        }
        if (eobrun_ > 0) {
            for (; k <= se; ++k) {
                int16_t &v = b[kNatural[k]];
                if (v != 0)
                    correct(v);
            }
            --eobrun_;
        }
    }

    size_t scan(const uint8_t *s, size_t sl, size_t pos)
    {
        if (comps_.empty())
            throw JpegError("scan before frame");
        if (sl < 1)
            throw JpegError("bad SOS");
        const int ns = s[0];
        if (ns < 1 || ns > 4 || sl < 4 + 2 * (size_t)ns)
            throw JpegError("bad SOS");
        std::vector<Component *> sc;
        for (int i = 0; i < ns; ++i) {
            Component *k = nullptr;
            for (Component &c : comps_)
                if (c.id == s[1 + 2 * i])
                    k = &c;
            if (!k)
                throw JpegError("scan names an unknown component");
            k->td = s[2 + 2 * i] >> 4;
            k->ta = s[2 + 2 * i] & 15;
            if (k->td > 3 || k->ta > 3)
                throw JpegError("bad table selector");
            sc.push_back(k);
        }
        const int ss = s[1 + 2 * ns], se = s[2 + 2 * ns], ah = s[3 + 2 * ns] >> 4, al = s[3 + 2 * ns] & 15;
        if (progressive_) {
            if (ss > se || se > 63 || (ss == 0 && se != 0) || (ss > 0 && ns != 1) || al > 13)
                throw JpegError("bad progressive scan parameters");
        }
        // jdhuff.c jpeg_make_d_derived_tbl: a table used for DC may only hold
        // magnitude categories 0..15 (a larger one would shift by >= 32 below)
        if (!progressive_ || (ss == 0 && ah == 0))
            for (Component *c : sc)
                if (dc_[c->td].present && dc_[c->td].max_sym > 15)
                    throw JpegError("bad Huffman table (DC symbol > 15)");
        for (Component *c : sc)
            c->pred = 0;
        eobrun_ = 0;
        BitReader br{d_, n_, pos};
        // non-interleaved scans cover ceil(dw/8) x ceil(dh/8) blocks, one block per MCU
        const bool single = ns == 1;
        const int mx = single ? (sc[0]->dw + 7) / 8 : mcux_, my = single ? (sc[0]->dh + 7) / 8 : mcuy_;
        const long total = (long)mx * my;
        int togo = restart_;
        for (long m = 0; m < total; ++m) {
            if (restart_ && togo == 0) {
                br.restart();
                for (Component *c : sc)
                    c->pred = 0;
                eobrun_ = 0;
                togo = restart_;
            }
            const int x = (int)(m % mx), y = (int)(m / mx);
            if (single) {
                Component &c = *sc[0];
                block(br, c, &c.coef[((size_t)y * c.bw + x) * 64], ss, se, ah, al);
            } else {
                for (Component *c : sc)
                    for (int by = 0; by < c->v; ++by)
                        for (int bx = 0; bx < c->h; ++bx) {
                            const size_t bi = (size_t)(y * c->v + by) * c->bw + (x * c->h + bx);
                            block(br, *c, &c->coef[bi * 64], ss, se, ah, al);
                        }
            }
            if (restart_)
                --togo;
        }
        any_scan_ = true;
        // the entropy-coded data ends at the next marker that is not RSTn
        size_t p = br.pos;
        while (p + 1 < n_) {
            if (d_[p] == 0xFF && d_[p + 1] != 0x00 && d_[p + 1] != 0xFF && !(d_[p + 1] >= 0xD0 && d_[p + 1] <= 0xD7))
                return p;
            ++p;
        }
        return n_;
    }

    Image finish()
    {
        for (Component &c : comps_) {
            const int stride = 8 * c.bw;
            c.plane.assign((size_t)stride * 8 * c.bh, 0);
            const int nbx = (c.dw + 7) / 8, nby = (c.dh + 7) / 8;
            for (int by = 0; by < nby; ++by)
                for (int bx = 0; bx < nbx; ++bx)
                    idct_islow(&c.coef[((size_t)by * c.bw + bx) * 64], q_[c.tq],
                               &c.plane[(size_t)by * 8 * stride + (size_t)bx * 8], stride);
            c.coef.clear();
            c.coef.shrink_to_fit();
        }
        Image im;
        im.width = width_;
        im.height = height_;
        im.bgr.resize((size_t)width_ * height_ * 3);
        const size_t np = (size_t)width_ * height_;
        if (comps_.size() == 1) { // IMREAD_COLOR of a gray JPEG: B = G = R
            const std::vector<uint8_t> g = upsample(comps_[0], hmax_, vmax_, width_, height_);
            for (size_t i = 0; i < np; ++i)
                im.bgr[3 * i] = im.bgr[3 * i + 1] = im.bgr[3 * i + 2] = g[i];
            return im;
        }
        std::vector<uint8_t> p[3];
        for (int c = 0; c < 3; ++c)
            p[c] = upsample(comps_[c], hmax_, vmax_, width_, height_);
        // jdapimin.c default_decompress_parms: JFIF -> YCbCr; Adobe transform 0 ->
        // RGB; component ids 'R','G','B' -> RGB; otherwise YCbCr
        bool rgb = false;
        if (!jfif_) {
            if (adobe_)
                rgb = adobe_transform_ == 0;
            else
                rgb = comps_[0].id == 'R' && comps_[1].id == 'G' && comps_[2].id == 'B';
        }
        if (adobe_ && adobe_transform_ == 2)
            throw JpegError("unsupported JPEG colour transform (YCCK)");
        if (rgb) {
            for (size_t i = 0; i < np; ++i) {
                im.bgr[3 * i] = p[2][i];
                im.bgr[3 * i + 1] = p[1][i];
                im.bgr[3 * i + 2] = p[0][i];
            }
            return im;
        }
        // jdcolor.c build_ycc_rgb_table / ycc_rgb_convert (SCALEBITS 16)
        static int cr_r[256], cb_b[256], cr_g[256], cb_g[256];
        static bool built = false;
        if (!built) {
            const long half = 1L << 15;
            auto fix = [](double x) { return (long)(x * 65536.0 + 0.5); };
            for (int i = 0; i < 256; ++i) {
                const long x = i - 128;
                cr_r[i] = (int)((fix(1.40200) * x + half) >> 16);
                cb_b[i] = (int)((fix(1.77200) * x + half) >> 16);
                cr_g[i] = (int)(-fix(0.71414) * x);
                cb_g[i] = (int)(-fix(0.34414) * x + half);
            }
            built = true;
        }
        for (size_t i = 0; i < np; ++i) {
            const int y = p[0][i], cb = p[1][i], cr = p[2][i];
            im.bgr[3 * i + 2] = clamp255(y + cr_r[cr]);
            im.bgr[3 * i + 1] = clamp255(y + ((cb_g[cb] + cr_g[cr]) >> 16));
            im.bgr[3 * i] = clamp255(y + cb_b[cb]);
        }
        return im;
    }
};

} // namespace

bool is_jpeg(const std::string &d) { return d.size() >= 3 && (uint8_t)d[0] == 0xFF && (uint8_t)d[1] == 0xD8 && (uint8_t)d[2] == 0xFF; }

Image decode_jpeg(const std::string &d, const std::string &path)
{
    try {
        return Decoder((const uint8_t *)d.data(), d.size()).run();
    } catch (const JpegError &e) {
        throw std::runtime_error(path + ": " + e.what());
    }
}

} // namespace dpio
