// oracle/ref/camera_driver.cpp -- TEST INFRASTRUCTURE (golden-vector generator).
//
// Compiled ONLY in this container against the reference's own camera.hpp
// (the interactive controls UpdateRotate / UpdateTranslateUV / UpdateFov,
// camera.hpp:33-65, driven by main.cpp:118-142's mouse callbacks), by
// oracle/ref/Makefile into oracle/_ref/camera_driver.  Never built or run on
// the GPU box.  argv[1]: ops file ("kind a b" per line: 0 = init eye/center/up
// from the next line, 1 = rotate(a, b), 2 = translate(a, b), 3 = fov(a));
// argv[2]: output, one line of 31 floats per op (eye center up fov aspect u v
// w distance lowerLeftCorner horizontal vertical).  The reference's own
// std::cout progress lines go to stdout and are ignored.
#include "model.hpp"     // completes the global std::vector<Light/Model> types of PnRT.hpp
#include "camera.hpp"

#include <cstdio>

int main(int argc, char** argv) {
    if (argc != 3) return 2;
    FILE* in = fopen(argv[1], "r");
    FILE* out = fopen(argv[2], "w");
    if (!in || !out) return 2;
    Camera cam;
    int kind;
    float a, b;
    while (fscanf(in, "%d %f %f", &kind, &a, &b) == 3) {
        if (kind == 0) {
            float e[3], c[3], u[3], fov, aspect;
            if (fscanf(in, "%f %f %f %f %f %f %f %f %f %f %f", &e[0], &e[1], &e[2], &c[0], &c[1], &c[2], &u[0], &u[1],
                       &u[2], &fov, &aspect) != 11)
                return 3;
            cam.UpdateCamera(glm::vec3(e[0], e[1], e[2]), glm::vec3(c[0], c[1], c[2]), glm::vec3(u[0], u[1], u[2]),
                             fov, aspect);
        } else if (kind == 1) {
            cam.UpdateRotate(a, b);
        } else if (kind == 2) {
            cam.UpdateTranslateUV(a, b);
        } else if (kind == 3) {
            cam.UpdateFov(a);
        }
        const glm::vec3* v[] = {&cam.eye, &cam.center, &cam.up};
        for (auto* p : v) fprintf(out, "%a %a %a ", (*p)[0], (*p)[1], (*p)[2]);
        fprintf(out, "%a %a ", cam.fov, cam.aspect);
        const glm::vec3* q[] = {&cam.u, &cam.v, &cam.w};
        for (auto* p : q) fprintf(out, "%a %a %a ", (*p)[0], (*p)[1], (*p)[2]);
        fprintf(out, "%a ", cam.distance);
        const glm::vec3* r[] = {&cam.lowerLeftCorner, &cam.horizontal, &cam.vertical};
        for (auto* p : r) fprintf(out, "%a %a %a ", (*p)[0], (*p)[1], (*p)[2]);
        fprintf(out, "\n");
    }
    fclose(out);
    return 0;
}
