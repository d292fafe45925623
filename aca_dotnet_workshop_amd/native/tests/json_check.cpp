// Conformance driver for native/src/json.hpp (tests/test_native_json.py): reads one JSON text per
// line (hex-encoded, so any byte can appear), parses it lax and strict and prints, per line,
// "<lax>\t<strict>" where each is the re-serialised value or "ERR".
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
    std::cout << run(view, false) << '\t' << run(view, true) << '\n';
  }
  return 0;
}
