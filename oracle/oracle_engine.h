/*
 * oracle_engine.h -- TEST INFRASTRUCTURE ONLY.  An independent restatement of
 * the per-(pixel, sample) engine specified in include/pt/pt_engine.h (the
 * reference DefaultRandomEngine recurrence 214013 v + 2531011, output v >> 32,
 * from a splitmix64-derived starting state), written
 * separately so that a bug in the product header cannot hide behind a shared
 * implementation.  tests/test_engine.py pins both against a pure-Python model.
 */
#ifndef PT_ORACLE_ENGINE_H
#define PT_ORACLE_ENGINE_H

#include <cstdint>

namespace oracle
{

inline uint64_t splitmix(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

/* Engine type satisfying the reference's T requirements
 * (include/path-trace.h:28-44: min(), max(), operator()). */
class SampleEngine
{
public:
    SampleEngine(uint64_t seed, uint64_t pixel, uint64_t sample)
    {
        uint64_t key = splitmix(seed) ^ (pixel << 20) ^ sample;
        s = splitmix(key);
    }
    static unsigned min() { return 0u; }
    static unsigned max() { return 0xFFFFFFFFu; }
    unsigned operator()()
    {
        s = 214013ull * s + 2531011ull; /* include/path-trace.h:45-49 */
        return (unsigned)(s >> 32);
    }
    uint64_t draws = 0; /* statistics only */
private:
    uint64_t s;
};

/* The reference's DefaultRandomEngine restated (include/path-trace.h:21-54):
 * 64-bit LCG 214013*v + 2531011, output v >> 32, seed(s): v = s ^ 0x12476242. */
class LcgEngine
{
public:
    explicit LcgEngine(unsigned seed) : v((uint64_t)(seed ^ 0x12476242u)) {}
    static unsigned min() { return 0u; }
    static unsigned max() { return 0xFFFFFFFFu; }
    unsigned operator()()
    {
        v = 214013ull * v + 2531011ull;
        return (unsigned)(v >> 32);
    }

private:
    uint64_t v;
};

} // namespace oracle

#endif
