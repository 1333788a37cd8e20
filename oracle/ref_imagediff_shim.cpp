// ORACLE (test infrastructure only): C entry points over the reference's own image
// comparison (renderer/util/ImageDiff.cpp, ImageDiff.cpp:94-372) and its vendored stb
// (renderer/ext/stb), compiled from the sources where they lie into
// oracle/_ref/libref_imagediff.so.  The reference instantiates stb inside
// TextureManager.cu (a CUDA file); this translation unit instantiates the same headers
// instead.  Used only to generate tests/golden/imagediff_ref.json and the diff images
// that pin vxpt_image_diff / vxpt_image_diff_png.
#define STB_IMAGE_IMPLEMENTATION
#include "ext/stb/stb_image.h"
#define STB_IMAGE_WRITE_IMPLEMENTATION
#include "ext/stb/stb_image_write.h"

#include "util/ImageDiff.h"

extern "C" {
// ImageDiff::compare(path, path); out: differentPixels, totalPixels, isIdentical, isVeryClose, isClose;
// fout: pixelDifferenceRatio, rmse, ssim
int ref_image_diff(const char *a, const char *b, int *out5, float *fout3) {
    const ImageDiffResult r = ImageDiff::compare(std::string(a), std::string(b));
    out5[0] = r.differentPixels;
    out5[1] = r.totalPixels;
    out5[2] = r.isIdentical;
    out5[3] = r.isVeryClose;
    out5[4] = r.isClose;
    fout3[0] = r.pixelDifferenceRatio;
    fout3[1] = r.rmse;
    fout3[2] = r.ssim;
    return 0;
}
// ImageDiff::generateDiffImage(path, path, out)
int ref_image_diff_png(const char *a, const char *b, const char *out) {
    return ImageDiff::generateDiffImage(std::string(a), std::string(b), std::string(out)) ? 0 : 1;
}
}
