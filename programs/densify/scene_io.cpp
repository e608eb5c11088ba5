// scene_io.cpp -- see scene_io.h.
#include "scene_io.h"

#include <zlib.h>

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace dpio {

// ---------------------------------------------------------------------------
// JSON (RFC 8259 subset sufficient for scene/settings files: no \u escapes
// beyond the BMP passthrough of ASCII)
// ---------------------------------------------------------------------------
const Json *Json::get(const std::string &k) const
{
    if (kind != Object)
        return nullptr;
    auto it = obj.find(k);
    return it == obj.end() ? nullptr : &it->second;
}

namespace {

struct Parser {
    const std::string &s;
    size_t i = 0;

    [[noreturn]] void fail(const char *what) const
    {
        throw std::runtime_error(std::string("JSON: ") + what + " at byte " + std::to_string(i));
    }
    void ws()
    {
        while (i < s.size() && std::isspace((unsigned char)s[i]))
            ++i;
    }
    bool eat(char c)
    {
        ws();
        if (i < s.size() && s[i] == c) {
            ++i;
            return true;
        }
        return false;
    }
    void expect(char c)
    {
        if (!eat(c))
            fail((std::string("expected '") + c + "'").c_str());
    }
    std::string string_lit()
    {
        ws();
        if (i >= s.size() || s[i] != '"')
            fail("expected string");
        ++i;
        std::string out;
        while (i < s.size() && s[i] != '"') {
            char c = s[i++];
            if (c == '\\') {
                if (i >= s.size())
                    fail("bad escape");
                const char e = s[i++];
                switch (e) {
                case 'n': out += '\n'; break;
                case 't': out += '\t'; break;
                case 'r': out += '\r'; break;
                case 'b': out += '\b'; break;
                case 'f': out += '\f'; break;
                case 'u': {
                    if (i + 4 > s.size())
                        fail("bad \\u escape");
                    const unsigned cp = (unsigned)std::strtoul(s.substr(i, 4).c_str(), nullptr, 16);
                    i += 4;
                    if (cp > 0x7f)
                        fail("non-ASCII \\u escape");
                    out += (char)cp;
                    break;
                }
                default: out += e; break; // \" \\ \/
                }
            } else {
                out += c;
            }
        }
        if (i >= s.size())
            fail("unterminated string");
        ++i;
        return out;
    }
    Json value()
    {
        ws();
        if (i >= s.size())
            fail("unexpected end");
        Json v;
        const char c = s[i];
        if (c == '{') {
            ++i;
            v.kind = Json::Object;
            if (eat('}'))
                return v;
            do {
                std::string k = string_lit();
                expect(':');
                v.obj[k] = value();
            } while (eat(','));
            expect('}');
        } else if (c == '[') {
            ++i;
            v.kind = Json::Array;
            if (eat(']'))
                return v;
            do {
                v.arr.push_back(value());
            } while (eat(','));
            expect(']');
        } else if (c == '"') {
            v.kind = Json::String;
            v.str = string_lit();
        } else if (s.compare(i, 4, "true") == 0) {
            v.kind = Json::Bool;
            v.b = true;
            i += 4;
        } else if (s.compare(i, 5, "false") == 0) {
            v.kind = Json::Bool;
            i += 5;
        } else if (s.compare(i, 4, "null") == 0) {
            i += 4;
        } else {
            const char *b = s.c_str() + i;
            char *e = nullptr;
            v.kind = Json::Number;
            v.num = std::strtod(b, &e);
            if (e == b)
                fail("bad value");
            i += (size_t)(e - b);
        }
        return v;
    }
};

} // namespace

Json parse_json(const std::string &text)
{
    Parser p{text};
    Json v = p.value();
    p.ws();
    if (p.i != text.size())
        p.fail("trailing characters");
    return v;
}

std::string read_file(const std::string &path)
{
    std::ifstream f(path, std::ios::binary);
    if (!f)
        throw std::runtime_error("cannot open " + path);
    std::ostringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

// ---------------------------------------------------------------------------
// images
// ---------------------------------------------------------------------------
namespace {

uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

int paeth(int a, int b, int c)
{
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

Image decode_png(const std::string &d, const std::string &path)
{
    const uint8_t *p = (const uint8_t *)d.data();
    size_t off = 8;
    int w = 0, h = 0, depth = 0, ctype = -1, interlace = 0;
    std::string idat;
    while (off + 12 <= d.size()) {
        const uint32_t len = be32(p + off);
        const std::string type((const char *)p + off + 4, 4);
        if (off + 12 + len > d.size())
            throw std::runtime_error(path + ": truncated PNG chunk");
        const uint8_t *c = p + off + 8;
        if (type == "IHDR") {
            w = (int)be32(c);
            h = (int)be32(c + 4);
            depth = c[8];
            ctype = c[9];
            interlace = c[12];
        } else if (type == "IDAT") {
            idat.append((const char *)c, len);
        } else if (type == "IEND") {
            break;
        }
        off += 12 + len;
    }
    const int ch = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 4 ? 2 : ctype == 6 ? 4 : 0;
    if (w <= 0 || h <= 0 || depth != 8 || ch == 0 || interlace != 0)
        throw std::runtime_error(path + ": unsupported PNG (need 8-bit gray/GA/RGB/RGBA, non-interlaced)");
    const size_t stride = (size_t)w * ch;
    std::vector<uint8_t> raw((stride + 1) * (size_t)h);
    uLongf rawlen = (uLongf)raw.size();
    if (uncompress(raw.data(), &rawlen, (const Bytef *)idat.data(), (uLong)idat.size()) != Z_OK ||
        rawlen != raw.size())
        throw std::runtime_error(path + ": corrupt PNG image data");
    std::vector<uint8_t> px(stride * (size_t)h);
    for (int y = 0; y < h; ++y) {
        const uint8_t f = raw[(stride + 1) * y];
        const uint8_t *src = &raw[(stride + 1) * y + 1];
        uint8_t *row = &px[stride * y];
        const uint8_t *up = y ? &px[stride * (y - 1)] : nullptr;
        for (size_t x = 0; x < stride; ++x) {
            const int a = x >= (size_t)ch ? row[x - ch] : 0;
            const int b = up ? up[x] : 0;
            const int cc = (up && x >= (size_t)ch) ? up[x - ch] : 0;
            int v = src[x];
            switch (f) {
            case 0: break;
            case 1: v += a; break;
            case 2: v += b; break;
            case 3: v += (a + b) >> 1; break;
            case 4: v += paeth(a, b, cc); break;
            default: throw std::runtime_error(path + ": bad PNG filter");
            }
            row[x] = (uint8_t)v;
        }
    }
    Image im;
    im.width = w;
    im.height = h;
    im.bgr.resize((size_t)w * h * 3);
    for (size_t i = 0; i < (size_t)w * h; ++i) {
        const uint8_t *s = &px[i * ch];
        uint8_t *o = &im.bgr[i * 3];
        if (ch >= 3) {
            o[0] = s[2];
            o[1] = s[1];
            o[2] = s[0];
        } else {
            o[0] = o[1] = o[2] = s[0];
        }
    }
    return im;
}

Image decode_ppm(const std::string &d, const std::string &path)
{
    std::istringstream in(d);
    std::string magic;
    in >> magic;
    auto num = [&]() {
        in >> std::ws;
        while (in.peek() == '#') {
            std::string line;
            std::getline(in, line);
            in >> std::ws;
        }
        int v = -1;
        in >> v;
        return v;
    };
    const int w = num(), h = num(), maxv = num();
    if (magic != "P6" || w <= 0 || h <= 0 || maxv != 255)
        throw std::runtime_error(path + ": unsupported PPM (need binary P6, maxval 255)");
    in.get();
    Image im;
    im.width = w;
    im.height = h;
    im.bgr.resize((size_t)w * h * 3);
    in.read((char *)im.bgr.data(), (std::streamsize)im.bgr.size());
    if ((size_t)in.gcount() != im.bgr.size())
        throw std::runtime_error(path + ": truncated PPM");
    for (size_t i = 0; i < im.bgr.size(); i += 3)
        std::swap(im.bgr[i], im.bgr[i + 2]); // RGB -> BGR
    return im;
}

} // namespace

Image load_image(const std::string &path)
{
    const std::string d = read_file(path);
    static const uint8_t png_sig[8] = {0x89, 'P', 'N', 'G', 0x0d, 0x0a, 0x1a, 0x0a};
    if (d.size() >= 8 && std::memcmp(d.data(), png_sig, 8) == 0)
        return decode_png(d, path);
    if (is_jpeg(d))
        return decode_jpeg(d, path);
    if (d.size() >= 2 && d[0] == 'P' && d[1] == '6')
        return decode_ppm(d, path);
    throw std::runtime_error(path + ": unsupported image format (JPEG, PNG or binary PPM)");
}

// ---------------------------------------------------------------------------
// scene / seeds / PLY
// ---------------------------------------------------------------------------
Scene read_scene(const std::string &path)
{
    const Json j = parse_json(read_file(path));
    const Json *ip = j.get("imagesPath");
    const Json *vs = j.get("views");
    if (!ip || ip->kind != Json::String || !vs || vs->kind != Json::Array)
        throw std::runtime_error(path + ": need \"imagesPath\" (string) and \"views\" (array)");
    Scene sc;
    sc.images_path = ip->str;
    for (const Json &v : vs->arr) {
        const Json *fn = v.get("filename");
        const Json *pm = v.get("projectionMatrix");
        if (!fn || fn->kind != Json::String || !pm || pm->kind != Json::Array || pm->arr.size() != 3)
            throw std::runtime_error(path + ": each view needs \"filename\" and a 3x4 \"projectionMatrix\"");
        SceneView sv;
        // stlplus::create_filespec(images_path, filename): directory + '/' + name
        sv.filename = sc.images_path.empty() ? fn->str
                      : (sc.images_path.back() == '/' ? sc.images_path + fn->str
                                                      : sc.images_path + "/" + fn->str);
        for (int r = 0; r < 3; ++r) {
            const Json &row = pm->arr[r];
            if (row.kind != Json::Array || row.arr.size() != 4)
                throw std::runtime_error(path + ": projectionMatrix rows must have 4 numbers");
            for (int c = 0; c < 4; ++c)
                sv.P[4 * r + c] = row.arr[c].num;
        }
        sc.views.push_back(sv);
    }
    return sc;
}

std::vector<double> read_seeds(const std::string &path)
{
    std::istringstream in(read_file(path));
    std::vector<double> xyz;
    std::string line;
    while (std::getline(in, line)) {
        const size_t h = line.find('#');
        if (h != std::string::npos)
            line.resize(h);
        std::istringstream ls(line);
        double x, y, z;
        if (ls >> x >> y >> z) {
            xyz.push_back(x);
            xyz.push_back(y);
            xyz.push_back(z);
        }
    }
    return xyz;
}

void write_ply(const std::string &path, const std::vector<CloudPoint> &pts)
{
    FILE *f = std::fopen(path.c_str(), "wb");
    if (!f)
        throw std::runtime_error("cannot write " + path);
    std::fprintf(f, "ply\nformat ascii 1.0\nelement vertex %zu\n", pts.size());
    std::fprintf(f, "property float x\nproperty float y\nproperty float z\n");
    std::fprintf(f, "property uchar red\nproperty uchar green\nproperty uchar blue\n");
    std::fprintf(f, "property float nx\nproperty float ny\nproperty float nz\nend_header\n");
    for (const CloudPoint &p : pts)
        std::fprintf(f, "%g %g %g %u %u %u %g %g %g\n", (double)p.pos[0], (double)p.pos[1], (double)p.pos[2],
                     (unsigned)p.rgb[0], (unsigned)p.rgb[1], (unsigned)p.rgb[2], (double)p.normal[0],
                     (double)p.normal[1], (double)p.normal[2]);
    if (std::fclose(f) != 0)
        throw std::runtime_error("write failed: " + path);
}

} // namespace dpio
