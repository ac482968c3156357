// DebuggingUtilities.hpp — drop-in for the reference include/DebuggingUtilities.hpp (a
// variadic print and the console colour codes).
#pragma once
#include <iostream>

namespace DebuggingUtilities {
inline void print() { std::cout << std::endl; }
template <typename T, typename... Args>
void print(T contents, Args... args) {
  std::cout << (contents) << " ";
  print(args...);
}
}  // namespace DebuggingUtilities

#define _NORMAL_ "\x1b[0m"
#define _BLACK_ "\x1b[30;47m"
#define _RED_ "\x1b[31;40m"
#define _GREEN_ "\x1b[32;40m"
#define _YELLOW_ "\x1b[33;40m"
#define _BLUE_ "\x1b[34;40m"
#define _MAGENTA_ "\x1b[35;40m"
#define _CYAN_ "\x1b[36;40m"
#define _WHITE_ "\x1b[37;40m"
