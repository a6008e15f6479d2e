// meduce-gpu: drop-in CLI for the reference binary (/root/reference/src/main.rs).
// Same input default ("shakes.txt" in the working directory, main.rs:10), same
// outputs: final_result.txt with "{word} {count}\n" lines (main.rs:170-182) and
// "Top 10 words:" + "{word}: {count}" on stdout (main.rs:184-192).  The hot
// section (main.rs:16-22) is one mox_count_file call on the GPU.  No
// intermediate map files exist, so the reference's cleanup lines
// ("Successfully deleted: ...", main.rs:194-202) are not printed.
// Exit status 1 with a message on stderr on any error, like `main` returning Err.
#include <cstdio>
#include <cstring>
#include <string>

#include "mox.h"

int main(int argc, char** argv) {
  std::string path = "shakes.txt", out = "final_result.txt";
  int device = -1;
  for (int i = 1; i < argc; i++) {
    if (!strcmp(argv[i], "--device") && i + 1 < argc) device = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--out") && i + 1 < argc) out = argv[++i];
    else path = argv[i];
  }
  mox_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.device = device;
  mox_engine* e = nullptr;
  if (mox_engine_create(&cfg, &e) != MOX_OK) { fprintf(stderr, "Error: %s\n", mox_last_error()); return 1; }
  mox_table* t = nullptr;
  int rc = mox_count_file(e, path.c_str(), &t);
  if (rc != MOX_OK) {
    fprintf(stderr, "Error: %s\n", mox_last_error());
    mox_engine_destroy(e);
    return 1;
  }
  rc = mox_write_final_result(t, out.c_str());
  if (rc == MOX_OK) rc = mox_print_top_words(t, 10);
  if (rc != MOX_OK) fprintf(stderr, "Error: %s\n", mox_last_error());
  mox_table_free(t);
  mox_engine_destroy(e);
  return rc == MOX_OK ? 0 : 1;
}
