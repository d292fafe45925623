// Conformance driver for native/src/json.hpp (tests/test_native_json.py): reads one JSON text per
// line (hex-encoded, so any byte can appear), parses it lax and strict and prints, per line,
// "<lax>\t<strict>\t<valid>\t<compact>": the re-serialised values or "ERR", tt::valid's verdict
// (1/0) and, for valid texts, the hex of tt::compact's output.
#include <cstdio>
#include <cstring>
#include <memory>
#include <iostream>
#include <string>

#include "json.hpp"

static std::string unhex(const std::string& h) {
  std::string out;
  for (size_t i = 0; i + 1 < h.size(); i += 2) out += (char)std::stoi(h.substr(i, 2), nullptr, 16);
  return out;
}

static std::string run(std::string_view text, bool strict) {
  try {
    tt::Value v = strict ? tt::parse_strict(text) : tt::parse(text);
    return tt::dump(v);
  } catch (const tt::ParseError&) {
    return "ERR";
  }
}

int main() {
  std::string line;
  while (std::getline(std::cin, line)) {
    // parse from an exactly sized heap copy, so ASan sees any read past the end of the text
    std::string text = unhex(line);
    std::unique_ptr<char[]> buf(new char[text.size() + (text.empty() ? 1 : 0)]);
    std::memcpy(buf.get(), text.data(), text.size());
    std::string_view view(buf.get(), text.size());
    const bool ok = tt::valid(view);
    std::string hex;
    if (ok) {
      static const char* d = "0123456789abcdef";
      for (unsigned char c : tt::compact(view)) hex += d[c >> 4], hex += d[c & 15];
    }
    std::cout << run(view, false) << '\t' << run(view, true) << '\t' << (ok ? 1 : 0) << '\t' << hex << '\n';
  }
  return 0;
}
