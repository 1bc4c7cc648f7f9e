/* devsrc.cpp -- the device library text (device/pt_device.h), embedded at
 * build time so every generated scene module carries the exact header the
 * library was built with (the JIT cache key hashes it). */
#include "internal.h"

namespace pt
{
std::string device_library_source()
{
    static const char src[] =
#include "pt_device_src.inc"
        ;
    return src;
}
std::string device_user_object_source()
{
    static const char src[] =
#include "pt_user_object_src.inc"
        ;
    return src;
}
} // namespace pt
