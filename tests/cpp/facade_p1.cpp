// Builds the north-star scene P1 (pathtrace/scenes.py scene_p1) with the C++
// facade include/pt/PathTrace.hpp, written the way the reference's demo
// builds its world (src/test.cpp:107-145), then
//   facade_p1 key DEPTH                 -> prints the scene's code-object key (no GPU)
//   facade_p1 render W H SPP DEPTH OUT  -> renders on device 0, writes W*H*3 f32 to OUT
//   facade_p1 errors                    -> checks the error mapping (no GPU)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>

#include "pt/PathTrace.hpp"

using namespace PathTrace;

int main(int argc, char **argv)
{
    if (argc < 2)
        return 2;
    Material diffuse(new ColorTexture(0.8f), new ColorTexture(1));
    Material mirror(new ColorTexture(0.99f), new ColorTexture(0));
    Material glass(new ColorTexture(0.7f), new ColorTexture(0), new ColorTexture(0), new ColorTexture(0.9f), 1.3f,
                   new ColorTexture(1));
    Material sky(new ColorTexture(0), new ColorTexture(0), new ColorTexture(0.5f, 0.7f, 1.0f));
    Object *left = new Difference(new Union(new Sphere(Vector3D(-1, 0, -4), .6f, &diffuse),
                                            new Sphere(Vector3D(-.5f, 0, -4), .6f, &diffuse)),
                                  new Sphere(Vector3D(-.7f, .3f, -3.6f), .4f, &diffuse));
    Object *right = new Difference(new Union(new Sphere(Vector3D(1, 0, -4), .6f, &glass),
                                             new Sphere(Vector3D(1.4f, .2f, -4.2f), .5f, &mirror)),
                                   new Sphere(Vector3D(1, 0, -3.4f), .3f, &glass));
    std::unique_ptr<Object> world(new Union(left, new Union(right, new Plane(Vector3D(0, 0, 1), 200, &sky))));

    try {
        if (!strcmp(argv[1], "errors")) {
            bool ok = false;
            try {
                invert(Matrix::scale(0.0f));
            } catch (std::domain_error &) {
                ok = true;
            }
            if (!ok)
                return 3;
            ok = false;
            try {
                Image("/nonexistent.hdr");
            } catch (ImageLoadError &) {
                ok = true;
            }
            if (!ok)
                return 4;
            Matrix r = Matrix::rotateY(0.5);
            Matrix id = r.concat(invert(r));
            printf("errors ok %.6f %.6f\n", id.x00, id.x11);
            return 0;
        }
        Renderer renderer(world.get());
        if (!strcmp(argv[1], "key") && argc == 3) {
            printf("%s\n", pt_scene_kernel_key(renderer.handle(), atoi(argv[2])));
            return 0;
        }
        if (!strcmp(argv[1], "render") && argc == 7) {
            Renderer::Settings st;
            st.width = atoi(argv[2]), st.height = atoi(argv[3]);
            st.sampleCount = atoi(argv[4]), st.rayDepth = atoi(argv[5]);
            std::vector<Color> img = renderer.render(st);
            FILE *f = fopen(argv[6], "wb");
            if (!f)
                return 5;
            fwrite(img.data(), sizeof(Color), img.size(), f);
            fclose(f);
            return 0;
        }
    } catch (std::exception &e) {
        fprintf(stderr, "facade_p1: %s\n", e.what());
        return 1;
    }
    return 2;
}
