// pcap2mgen -- the reference's offline tool (src/common/pcap2mgen.cpp) on the GPU.
//
// Same command set and matching rules as the reference's ProcessCommands / GetCmdType
// (:25-248): report, analytic, infile <f>, outfile <f>, trace, rxlog on|off, flush,
// window <sec> -- given bare, as there (the table's +/- only says whether an argument
// follows), each matched case-insensitively by a unique prefix; stdin / stdout by default.
// The whole capture is read, decoded on the device by mgenx::Pcap2Mgen
// (include/mgenx_pcap.hpp) and the log written in one piece.  "trace" (MAC addresses in
// front of each line) is not supported and is reported as such; "flush" has nothing to do
// here.  Extra: "epoch" selects epoch timestamps (Mgen::SetEpochTimestamp).
#include <ctype.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "mgenx_pcap.hpp"

namespace {

enum CmdType { CMD_INVALID, CMD_ARG, CMD_NOARG };
const char* const kCmds[] = {"-report", "-analytic", "+infile", "+outfile", "-trace",
                             "+rxlog",  "-flush",    "+window", "-epoch",   nullptr};

// GetCmdType (:71-109): a unique case-insensitive prefix match
CmdType GetCmdType(const char* cmd, const char** which) {
  if (!cmd) return CMD_INVALID;
  std::string low;
  for (const char* p = cmd; *p && low.size() < 31; p++) low += (char)tolower(*p);
  CmdType type = CMD_INVALID;
  bool matched = false;
  for (const char* const* c = kCmds; *c; c++) {
    if (!strncmp(low.c_str(), *c + 1, low.size())) {
      if (matched) return CMD_INVALID;  // ambiguous
      matched = true;
      type = ('+' == (*c)[0]) ? CMD_ARG : CMD_NOARG;
      *which = *c + 1;
    }
  }
  return type;
}

bool ReadAll(FILE* f, std::vector<uint8_t>& out) {
  uint8_t buf[1 << 16];
  size_t k;
  while ((k = fread(buf, 1, sizeof(buf), f)) > 0) out.insert(out.end(), buf, buf + k);
  return !ferror(f);
}

}  // namespace

int main(int argc, char* argv[]) {
  mgenx::PcapOptions opt;
  FILE* infile = stdin;
  FILE* outfile = stdout;
  for (int i = 1; i < argc;) {
    const char* which = nullptr;
    const CmdType t = GetCmdType(argv[i], &which);
    if (t == CMD_INVALID) {
      fprintf(stderr, "pcap2mgen error: invalid command: %s\n", argv[i]);
      return -1;
    }
    const char* val = (t == CMD_ARG && i + 1 < argc) ? argv[i + 1] : nullptr;
    if (t == CMD_ARG && !val) {
      fprintf(stderr, "pcap2mgen ProcessCommands(%s) missing argument\n", argv[i]);
      return -1;
    }
    if (!strcmp(which, "analytic") || !strcmp(which, "report")) {
      opt.analytics = true;
    } else if (!strcmp(which, "infile")) {
      if (!(infile = fopen(val, "rb"))) {
        fprintf(stderr, "pcap2mgen: error opening input file: %s", val);
        return -1;
      }
    } else if (!strcmp(which, "outfile")) {
      if (!(outfile = fopen(val, "w+"))) {
        fprintf(stderr, "pcap2mgen: error opening output file: %s", val);
        return -1;
      }
    } else if (!strcmp(which, "trace")) {
      fprintf(stderr, "pcap2mgen: trace (MAC address prefix) is not supported\n");
      return -1;
    } else if (!strcmp(which, "rxlog")) {
      std::string v;
      for (const char* p = val; *p && v.size() < 4; p++) v += (char)tolower(*p);
      if (!v.empty() && !strncmp("on", v.c_str(), v.size())) opt.log_rx = true;
      else if (!v.empty() && !strncmp("off", v.c_str(), v.size())) opt.log_rx = false;
      else {
        fprintf(stderr, "pcap2mgen OnCommand Error: wrong argument to rxlog: %s\n", val);
        return -1;
      }
    } else if (!strcmp(which, "window")) {
      double w;
      if (1 != sscanf(val, "%lf", &w) || w <= 0.0)
        fprintf(stderr, "Mgen::OnCommand() Error: invalid WINDOW interval\n");
      else
        opt.window = w;
    } else if (!strcmp(which, "epoch")) {
      opt.epoch = true;
    }  // flush: nothing to do
    i += (t == CMD_ARG) ? 2 : 1;
  }
  std::vector<uint8_t> file;
  if (!ReadAll(infile, file)) {
    perror("pcap2mgen: read error");
    return -1;
  }
  try {
    mgenx::Context ctx(0);
    mgenx::Pcap2Mgen p(ctx, opt);
    const std::string log = p.Run(file.data(), file.size());
    if (!log.empty() && fwrite(log.data(), 1, log.size(), outfile) != log.size()) {
      perror("pcap2mgen: write error");
      return -1;
    }
  } catch (const std::exception& e) {
    fprintf(stderr, "pcap2mgen: %s\n", e.what());
    return -1;
  }
  if (infile != stdin) fclose(infile);
  if (outfile != stdout) fclose(outfile);
  return 0;
}
