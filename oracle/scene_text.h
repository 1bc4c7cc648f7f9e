/*
 * scene_text.h -- TEST INFRASTRUCTURE ONLY (oracle/).  Parser for the plain-text
 * scene description shared by the CPU oracle (oracle/oracle.cpp) and the
 * reference driver (oracle/ref_driver.cpp).  Never linked into the product.
 *
 * One item per line, whitespace separated; floats are C99 hex floats (or any
 * strtof-parsable text), so both parsers see bit-identical inputs.  Ids refer
 * to earlier lines of the same kind.  The constructors mirrored are the
 * reference's public scene API:
 *
 *   image <id> raw <w> <h> <path>          RGBA f32 little-endian, row 0 = top
 *   image <id> hdr <path>                  Radiance .hdr (reference src/image.cpp:83-324)
 *   tex <id> color <r> <g> <b>             ColorTexture          include/texture.h:29-58
 *   tex <id> image <img>                   ImageTexture          include/image_texture.h:9-33
 *   tex <id> image_alpha <img>             ImageAlphaTexture     include/image_texture.h:35-70
 *   tex <id> skybox <t> <b> <l> <r> <f> <k> ImageSkyboxTexture   include/image_texture.h:72-115
 *   tex <id> skybox_alpha <6 imgs>         ImageSkyboxAlphaTexture include/image_texture.h:117-181
 *   tex <id> multiply <r> <g> <b> <tex>    MultiplyTexture       include/filter_texture.h:36-56
 *   tex <id> log <tex>                     LogTexture            include/filter_texture.h:58-82
 *   tex <id> mirrorball <tex>              MirrorBallSkymapTexture include/transform_texture.h:33-59
 *   tex <id> spherical <tex>               SphericalCoordinatesSkymapTexture :61-85
 *   tex <id> xform <12 f> <tex>            TransformedTexture    include/texture.h:60-90
 *   tex <id> coord                         test-only: getColor(v) = v (pins coordinate maps)
 *   tex <id> user <slot> <n> <n f>         a user Texture subclass: the host functions registered
 *                                          for <slot> (oracle_register_user_texture), n parameters
 *   mat <id> <refl> <scat> <emis> <trans> <ior> <trc>   Material include/material.h:10-37
 *   obj <id> sphere <cx> <cy> <cz> <r> <mat>             Sphere   src/sphere.cpp:6-12
 *   obj <id> plane <nx> <ny> <nz> <d> <mat>              Plane    src/plane.cpp:6-9
 *   obj <id> union|intersection|difference <a> <b>       src/{union,intersection,difference}.cpp
 *   obj <id> xform <12 f> <child>                        TransformedObject include/object.h:26-98
 *   obj <id> user <slot> <mat> <n> <n f>                 a user Object subclass: the host functions
 *                                                        registered for <slot> (oracle_register_user_object)
 *   root <id>
 *
 * Matrices use the reference constructor order (x00 x10 x20 x30 x01 ... x32),
 * include/transform.h:148-174.
 */
#ifndef PT_ORACLE_SCENE_TEXT_H
#define PT_ORACLE_SCENE_TEXT_H

#include <cstdlib>
#include <cstring>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace scenetext
{

struct Item
{
    std::string kind;  // "image" | "tex" | "mat" | "obj" | "root"
    std::string type;  // e.g. "sphere", "color", "raw"
    int id = -1;
    std::vector<float> f;  // float operands in order
    std::vector<int> i;    // integer operands (ids, dims) in order
    std::string path;
};

struct Desc
{
    std::vector<Item> images, textures, materials, objects;
    int root = -1;
};

inline float parse_float(const std::string &s)
{
    char *end = nullptr;
    float v = std::strtof(s.c_str(), &end);
    if (end == s.c_str() || *end != '\0')
        throw std::runtime_error("scene_text: bad float '" + s + "'");
    return v;
}

inline int parse_int(const std::string &s)
{
    char *end = nullptr;
    long v = std::strtol(s.c_str(), &end, 10);
    if (end == s.c_str() || *end != '\0')
        throw std::runtime_error("scene_text: bad int '" + s + "'");
    return (int)v;
}

inline Desc parse(const std::string &text)
{
    Desc d;
    std::istringstream in(text);
    std::string line;
    while (std::getline(in, line)) {
        std::istringstream ls(line);
        std::vector<std::string> tok;
        std::string t;
        while (ls >> t)
            tok.push_back(t);
        if (tok.empty() || tok[0][0] == '#')
            continue;
        Item it;
        it.kind = tok[0];
        if (it.kind == "root") {
            d.root = parse_int(tok.at(1));
            continue;
        }
        it.id = parse_int(tok.at(1));
        it.type = tok.at(2);
        auto need = [&](size_t n) {
            if (tok.size() != n)
                throw std::runtime_error("scene_text: wrong operand count in '" + line + "'");
        };
        if (it.kind == "image") {
            if (it.type == "raw") {
                need(6);
                it.i = {parse_int(tok[3]), parse_int(tok[4])};
                it.path = tok[5];
            } else if (it.type == "hdr") {
                need(4);
                it.path = tok[3];
            } else
                throw std::runtime_error("scene_text: unknown image kind " + it.type);
            d.images.push_back(it);
        } else if (it.kind == "tex") {
            const std::string &ty = it.type;
            if (ty == "color") {
                need(6);
                for (int k = 3; k < 6; k++) it.f.push_back(parse_float(tok[k]));
            } else if (ty == "image" || ty == "image_alpha" || ty == "log" || ty == "mirrorball" ||
                       ty == "spherical") {
                need(4);
                it.i = {parse_int(tok[3])};
            } else if (ty == "skybox" || ty == "skybox_alpha") {
                need(9);
                for (int k = 3; k < 9; k++) it.i.push_back(parse_int(tok[k]));
            } else if (ty == "multiply") {
                need(7);
                for (int k = 3; k < 6; k++) it.f.push_back(parse_float(tok[k]));
                it.i = {parse_int(tok[6])};
            } else if (ty == "xform") {
                need(16);
                for (int k = 3; k < 15; k++) it.f.push_back(parse_float(tok[k]));
                it.i = {parse_int(tok[15])};
            } else if (ty == "coord") {
                need(3);
            } else if (ty == "user") {
                if (tok.size() < 5)
                    throw std::runtime_error("scene_text: wrong operand count in '" + line + "'");
                it.i = {parse_int(tok[3]), parse_int(tok[4])};
                need(5 + (size_t)it.i[1]);
                for (size_t k = 5; k < tok.size(); k++) it.f.push_back(parse_float(tok[k]));
            } else
                throw std::runtime_error("scene_text: unknown texture " + ty);
            d.textures.push_back(it);
        } else if (it.kind == "mat") {
            // mat <id> <refl> <scat> <emis> <trans> <ior> <trc>
            tok.insert(tok.begin() + 2, "material");
            it.type = "material";
            need(9);
            it.i = {parse_int(tok[3]), parse_int(tok[4]), parse_int(tok[5]), parse_int(tok[6]),
                    parse_int(tok[8])};
            it.f = {parse_float(tok[7])};
            d.materials.push_back(it);
        } else if (it.kind == "obj") {
            const std::string &ty = it.type;
            if (ty == "sphere") {
                need(8);
                for (int k = 3; k < 7; k++) it.f.push_back(parse_float(tok[k]));
                it.i = {parse_int(tok[7])};
            } else if (ty == "plane") {
                need(8);
                for (int k = 3; k < 7; k++) it.f.push_back(parse_float(tok[k]));
                it.i = {parse_int(tok[7])};
            } else if (ty == "union" || ty == "intersection" || ty == "difference") {
                need(5);
                it.i = {parse_int(tok[3]), parse_int(tok[4])};
            } else if (ty == "xform") {
                need(16);
                for (int k = 3; k < 15; k++) it.f.push_back(parse_float(tok[k]));
                it.i = {parse_int(tok[15])};
            } else if (ty == "user") {
                if (tok.size() < 6)
                    throw std::runtime_error("scene_text: wrong operand count in '" + line + "'");
                it.i = {parse_int(tok[4]), parse_int(tok[3]), parse_int(tok[5])}; /* mat, slot, n */
                need(6 + (size_t)it.i[2]);
                for (size_t k = 6; k < tok.size(); k++) it.f.push_back(parse_float(tok[k]));
            } else
                throw std::runtime_error("scene_text: unknown object " + ty);
            d.objects.push_back(it);
        } else
            throw std::runtime_error("scene_text: unknown line kind " + it.kind);
    }
    if (d.root < 0)
        throw std::runtime_error("scene_text: no root");
    return d;
}

template <class V>
inline const Item &find(const V &v, int id, const char *what)
{
    for (const Item &it : v)
        if (it.id == id)
            return it;
    throw std::runtime_error(std::string("scene_text: unknown ") + what + " id " + std::to_string(id));
}

} // namespace scenetext

#endif
