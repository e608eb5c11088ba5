// scene_io.h -- host-side IO of the densify CLI: a small JSON reader (scene and
// settings files), JPEG/PNG/PPM image decoding to BGR8, seed files and the ASCII
// PLY writer.  Restates the reference's modules/io surface:
//   scene JSON  modules/io/json_reader.cpp:9-28 ({"imagesPath", "views": [{
//               "filename", "projectionMatrix": 3x4}]})
//   images      cv::imread BGR8 (modules/core/types.cpp:7-11)
//   point cloud PMVS::PrintCloud (methods/pmvs/utils.cpp:9-50): ASCII PLY,
//               x y z red green blue nx ny nz
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace dpio {

// ---- JSON -------------------------------------------------------------------
struct Json {
    enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
    bool b = false;
    double num = 0.0;
    std::string str;
    std::vector<Json> arr;
    std::map<std::string, Json> obj;

    const Json *get(const std::string &k) const;
};

// Parses `text`; throws std::runtime_error with the byte offset on bad input.
Json parse_json(const std::string &text);
std::string read_file(const std::string &path);

// ---- images -----------------------------------------------------------------
struct Image {
    int width = 0, height = 0;
    std::vector<uint8_t> bgr; // rows of 3*width bytes, B G R as cv::imread returns
};

// JPEG (baseline / extended sequential / progressive Huffman, 8-bit gray or
// YCbCr/RGB, EXIF orientation applied; jpeg.cpp), PNG (8-bit gray / gray+alpha
// / RGB / RGBA, non-interlaced) or binary PPM (P6, maxval 255); chosen by the
// file's signature.  Throws on anything else.
Image load_image(const std::string &path);

// the JPEG decoder behind load_image (cv::imread IMREAD_COLOR semantics)
bool is_jpeg(const std::string &data);
Image decode_jpeg(const std::string &data, const std::string &path);

// ---- scene ------------------------------------------------------------------
struct SceneView {
    std::string filename; // imagesPath joined with the view's filename
    double P[12];         // projectionMatrix, row-major
};

struct Scene {
    std::string images_path;
    std::vector<SceneView> views;
};

Scene read_scene(const std::string &path);

// ---- seeds / cloud ----------------------------------------------------------
// ASCII "x y z" per line ('#' comments allowed) -> xyz triples
std::vector<double> read_seeds(const std::string &path);

struct CloudPoint {
    float pos[3];
    uint8_t rgb[3];
    float normal[3];
};

// ASCII PLY exactly as PrintCloud writes it (%g floats, uchar colours)
void write_ply(const std::string &path, const std::vector<CloudPoint> &pts);

} // namespace dpio
