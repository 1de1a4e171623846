// libslu_mi355x_metis.so only: the error sink csrc/ordering.cpp reports to
// (in the other libraries it is the engine's slu_last_error string).
#include <cstdio>
#include <string>

namespace slu {
void set_last_error(const std::string &s) { fprintf(stderr, "METIS_NodeND (MI355X library): %s\n", s.c_str()); }
} // namespace slu
