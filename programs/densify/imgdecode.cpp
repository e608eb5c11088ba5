// imgdecode -- decode one image with the densify CLI's ingest (load_image:
// JPEG / PNG / PPM -> BGR8, as cv::imread IMREAD_COLOR) and write it as a
// binary PPM (RGB) to the output path; used by the CPU ingest tests.
//   imgdecode in.jpg out.ppm
#include "scene_io.h"

#include <cstdio>
#include <exception>

int main(int argc, char **argv)
{
    if (argc != 3) {
        std::fprintf(stderr, "usage: imgdecode <image> <out.ppm>\n");
        return 2;
    }
    try {
        const dpio::Image im = dpio::load_image(argv[1]);
        std::FILE *f = std::fopen(argv[2], "wb");
        if (!f) {
            std::fprintf(stderr, "cannot write %s\n", argv[2]);
            return 1;
        }
        std::fprintf(f, "P6\n%d %d\n255\n", im.width, im.height);
        for (size_t i = 0; i < im.bgr.size(); i += 3) {
            const unsigned char rgb[3] = {im.bgr[i + 2], im.bgr[i + 1], im.bgr[i]};
            std::fwrite(rgb, 1, 3, f);
        }
        std::fclose(f);
    } catch (const std::exception &e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
