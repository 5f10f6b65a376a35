// cg_parse.h -- node/cron spec parser on the host (parser.go:78-377), and
// Every (constantdelay.go:14-21).
#pragma once
#include <stdint.h>

#include <string>
#include <string_view>

namespace cg {

// ParseOption bits, parser.go:17-26
enum : int {
  OPT_SECOND = 1,
  OPT_MINUTE = 2,
  OPT_HOUR = 4,
  OPT_DOM = 8,
  OPT_MONTH = 16,
  OPT_DOW = 32,
  OPT_DOW_OPTIONAL = 64,
  OPT_DESCRIPTOR = 128,
};

constexpr uint64_t kStarBit = 1ULL << 63;  // spec.go:48-51

struct Schedule {
  int kind = 0;  // 0 *SpecSchedule, 1 ConstantDelaySchedule
  uint64_t second = 0, minute = 0, hour = 0, dom = 0, month = 0, dow = 0;
  int64_t delay_ns = 0;
};

// Parser{options}.Parse(spec).  0 = ok, -1 = error (err holds Go's message),
// -2 = the spec is empty (Go indexes spec[0] and panics; JobRule.Valid
// returns ErrNilRule before that, job.go:297-299).
int parse(int options, std::string_view spec, Schedule* out, std::string* err);
int get_range(std::string_view expr, unsigned min, unsigned max, int names, uint64_t* bits,
              std::string* err);
int get_field(std::string_view expr, unsigned min, unsigned max, int names, uint64_t* bits,
              std::string* err);
uint64_t get_bits(unsigned min, unsigned max, unsigned step);
int parse_duration(std::string_view s, int64_t* out, std::string* err);
int64_t every(int64_t d_ns);

}  // namespace cg
